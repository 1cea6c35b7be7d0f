mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_edge_slope.py tests/test_gpu_alexandridis.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_edge.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_edge.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/bench_edge.json 2> gpurun_out/bench_edge.err
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --slope-layout planes > gpurun_out/bench_planes.json 2> gpurun_out/bench_planes.err
