set -e
mkdir -p gpurun_out/r01am
timeout -k 10 500 python -m pytest tests/test_mesh.py -m gpu -x -q > gpurun_out/r01am/mtests.log 2>&1
timeout -k 10 200 python bench.py --scene mesh --no-cpu-baseline >> gpurun_out/r01am/bench_mesh.log 2>/dev/null
timeout -k 10 200 python bench.py --scene mesh --no-cpu-baseline --tune mesh_lds_stack=12 >> gpurun_out/r01am/bench_mesh.log 2>/dev/null
timeout -k 10 300 python bench.py --scene mixed --no-cpu-baseline --steps 2 --warmup 1 >> gpurun_out/r01am/bench_mixed.log 2>/dev/null
