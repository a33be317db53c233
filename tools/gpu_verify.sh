set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r01_gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r01_bench.json 2> gpurun_out/r01_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/r01_prof_bench.log 2>&1
