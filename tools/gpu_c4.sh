set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "flow_cancel or config4 or v4" > gpurun_out/r02q_tests.log 2>&1 || { tail -30 gpurun_out/r02q_tests.log; exit 1; }
tail -2 gpurun_out/r02q_tests.log
bash tools/xp_run.sh r02q "libgome_base.so libgome.so" "config4"
