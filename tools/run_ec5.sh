set -o pipefail
mkdir -p gpurun_out/ec5
timeout -k 10 500 python -u -m pytest tests/test_ecdsa_batch.py tests/test_ecdsa_der_gpu.py tests/test_gpu_verify_service.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/ec5/t.log 2>&1
rc=$?
tail -n 4 gpurun_out/ec5/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ecdsa_kernel_tput.py 4096 16384 32768 65536 131072 199680 262144 1048576 > gpurun_out/ec5/tput.log 2>&1 || exit 1
grep -v rows gpurun_out/ec5/tput.log | cut -c1-120
bash tools/gpu_check.sh ibd ibd4 50 14
