set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 -k "attention" > gpurun_out/t_attn.log 2>&1; rc=$?; tail -3 gpurun_out/t_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/attn_bench.py --modes 0,2 || exit $?
timeout -k 10 200 python tools/attn_bench.py --modes 0,2 --bidir || exit $?
