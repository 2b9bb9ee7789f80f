"""Copy the small text artefacts of GPU runs that DESIGN.md cites from gpurun_out/ (git-ignored
scratch) into profiles/evidence/<run>/, so the evidence is in history: test logs, bench lines,
rocprofv3 kernel-stats summaries.  Large traces (per-dispatch CSVs) stay behind.

  python tools/archive_evidence.py RUN [RUN ...]"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEEP = (".txt", ".jsonl", ".json", ".log", ".md")
MAX = 256 << 10

for run in sys.argv[1:]:
    src = os.path.join(ROOT, "gpurun_out", run)
    if not os.path.isdir(src):
        print("missing", run)
        continue
    n = 0
    for dp, _, files in os.walk(src):
        for f in files:
            p = os.path.join(dp, f)
            if not (f.endswith(KEEP) or f.endswith("_stats.csv")) or os.path.getsize(p) > MAX:
                continue
            dst = os.path.join(ROOT, "profiles", "evidence", run, os.path.relpath(p, src))
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copyfile(p, dst)
            n += 1
    print(run, n, "files")
