set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_solver_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "period_lane" > gpurun_out/pltest.log 2>&1
rc=$?
echo "test rc $rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then timeout -k 10 300 python -u tools/pl_probe.py > gpurun_out/plprobe.log 2>&1; echo "probe rc $?"; fi
