# single-level split rule: Hector parity, then c2 and north-star bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/c2s
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hector_gpu.py tests/test_ingest_gpu.py tests/test_backend_gpu.py > gpurun_out/c2s/test.log 2>&1 || { echo "FAIL test"; tail -30 gpurun_out/c2s/test.log; exit 1; }
tail -2 gpurun_out/c2s/test.log
timeout -k 10 300 python3 bench.py --config c2 > gpurun_out/c2s/c2.json 2> gpurun_out/c2s/c2.err || { echo "FAIL c2"; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/c2s/ns.json 2> gpurun_out/c2s/ns.err || { echo "FAIL ns"; exit 1; }
for f in c2 ns; do python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], r['read_only_frac'], d['pose_vs_ref']['vs_oracle_tree_order_exact_frac'])" gpurun_out/c2s/$f.json $f; done
