#!/bin/bash
# Round-6 GPU session A: every GPU test (failures do not stop the session; a crash or timeout does),
# A/B of the mixed solve's handoff variants and of the lsolve steering branch, the sharded bench
# path on one GPU (two gloo ranks sharing cuda:0 vs world 1), then the default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }   # pytest: 1 = test failures (keep going)
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -rf > $O/gputests.log 2>&1
rc=$?; echo "gputests rc $rc"; ok $rc || exit $rc
: > $O/ab_mixed.log
for L in "" libkmpc_h0.so libkmpc_h1.so libkmpc_ns.so; do
  echo "== ${L:-libkmpc.so}" >> $O/ab_mixed.log
  KMPC_DEV_LIB=$L REPS=3 NCHK=64 timeout -k 10 240 python3 -u tools/mixed_probe.py 65536 5e-5 >> $O/ab_mixed.log 2>&1 || exit $?
done
LIBS="libkmpc.so libkmpc_ns.so" SHAPES="N=64,H=10|N=30,H=5,cost|C1-shape|N=120,H=10|N=90,H=7|N=200,H=10|N=250,H=10" \
  timeout -k 10 400 bash tools/ab_shapes.sh || exit $?
timeout -k 10 300 python -u bench.py --global-windows 262144 --headline-only --cpu-seconds 0 --steps 2 --warmup 1 \
  --dump-w0 $O/w0_world1.npy > $O/shard_world1.log 2>&1 || exit $?
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --global-windows 262144 --backend gloo --share-device --headline-only \
  --cpu-seconds 0 --steps 2 --warmup 1 --dump-w0 $O/w0_world2.npy > $O/shard_world2.log 2>&1 || exit $?
python - > $O/shard_compare.log 2>&1 <<'EOF'
import numpy as np
a = np.load("gpurun_out/w0_world1.npy"); b = np.load("gpurun_out/w0_world2.npy")
print("shapes", a.shape, b.shape, "bit-identical", bool(np.array_equal(a, b)), "max|d|", float(np.abs(a - b).max()))
EOF
rm -f $O/w0_world1.npy $O/w0_world2.npy
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
echo "exit 0"
