#!/bin/bash
# Variant library for GPU A/B (run here, on the CPU): the product objects with some translation units
# rebuilt with extra flags, linked to koopman_mpc_portfolio_rebalancing_amd/libkmpc_NAME.so.
#   bash tools/build_var.sh NAME "FLAGS" TU[:OPT] ...      e.g. bash tools/build_var.sh h0 -DX=0 kmpc_solve_c3:-O2
set -e
cd "$(dirname "$0")/../koopman_mpc_portfolio_rebalancing_amd/csrc"
NAME=$1; FLAGS=$2; shift 2
make -s -j8 > /dev/null
mkdir -p _obj_$NAME
objs=""
pids=""
for spec in "$@"; do
  tu=${spec%%:*}; opt=-Os; [ "$spec" != "$tu" ] && opt=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable $opt $FLAGS \
    -c $tu.hip -o _obj_$NAME/$tu.o &
  pids="$pids $!"
  objs="$objs $tu"
done
for p in $pids; do wait $p; done
link=""
for o in _obj/*.o; do
  b=$(basename $o .o)
  if [[ " $objs " == *" $b "* ]]; then link="$link _obj_$NAME/$b.o"; else link="$link $o"; fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../libkmpc_$NAME.so $link
echo "built libkmpc_$NAME.so ($objs)"
