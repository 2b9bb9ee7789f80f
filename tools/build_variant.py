"""Build an experimental variant of libgome.so (tuning only; the product is gome_amd/libgome.so).

  python tools/build_variant.py TAG [ENV=VALUE ...] [-DMACRO ...]

ENV=VALUE pairs go to gen_plan_asm.py (e.g. GOME_PLAN_PF=4096); -D flags to hipcc.  Writes
gome_amd/libgome_TAG.so; load it with GOME_LIB=gome_amd/libgome_TAG.so."""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gome_amd import build  # noqa: E402

tag = sys.argv[1]
env = dict(os.environ)
defs = []
for a in sys.argv[2:]:
    if a.startswith("-D"):
        defs.append(a)
    else:
        k, v = a.split("=", 1)
        env[k] = v
tmp = tempfile.mkdtemp(prefix=f"gv_{tag}_")
shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
shutil.copytree(build.CSRC, os.path.join(tmp, "gome_amd", "csrc"))
csrc = os.path.join(tmp, "gome_amd", "csrc")
subprocess.run([sys.executable, os.path.join(csrc, "gen_plan_asm.py"), "--out", os.path.join(csrc, "flow_plan_asm.inc")],
               env=env, check=True)
out = os.path.join(build.PKG, f"libgome_{tag}.so")
srcs = [os.path.join(csrc, os.path.basename(s)) for s in build.SOURCES]
cmd = [build.HIPCC, f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", *build.DEVICE_FLAGS,
       *defs, "-I", os.path.join(tmp, "include"), *srcs, "-o", out]
subprocess.run(cmd, check=True)
shutil.rmtree(tmp)
print(out)
