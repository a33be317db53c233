export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "icp or registration" > gpurun_out/q_tests.log 2>&1; rc=$?; tail -3 gpurun_out/q_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_icp -o run --output-format csv -- python tools/prof_kernels.py icp_loop > gpurun_out/picp.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/qb.json 2>gpurun_out/qb.err; grep -o "\"icp\": {[^}]*}" gpurun_out/qb.json; grep -o "\"icp_30\": [0-9.]*" gpurun_out/qb.json
