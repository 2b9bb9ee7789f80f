set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/xp1
for L in libgome.so libgome_addonly.so; do
  echo "== $L"
  GOME_LIB=gome_amd/$L timeout -k 10 200 python -u tools/ubench_fc_plan.py 2>&1 | grep -v amdgpu.ids || exit 1
  GOME_LIB=gome_amd/$L timeout -k 10 200 python -u bench.py --steps 10 --e2e-steps 0 --no-cpu-baseline > gpurun_out/xp1/b_$L.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/xp1/b_$L.json'));print(d['value'],d['hot_book'])"
done
