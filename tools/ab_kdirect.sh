set -o pipefail
mkdir -p gpurun_out; : > gpurun_out/abk.log
for L in libkmpc_old.so libkmpc.so libkmpc_old.so libkmpc.so; do
  for S in "4096 30" "65536 10"; do set -- $S
    echo "== $L B=$1 N=$2" >> gpurun_out/abk.log
    KMPC_DEV_LIB=$L B=$1 N=$2 timeout -k 10 120 python3 -u tools/c2_graph_probe.py >> gpurun_out/abk.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rollout_gpu.py tests/test_window_gpu.py tests/test_dmd.py tests/test_backtest_gpu.py > gpurun_out/abk_tests.log 2>&1
