set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --no-sweep"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
for v in "c3 rt_fuse_shadows=1" "c3 rt_fuse_shadows=0" "c3 rt_fuse_shadows=1" "c3 rt_fuse_shadows=0" "c4 rt_fuse_shadows=1" "c4 rt_fuse_shadows=0"; do
  set -- $v; n=$1_${2//=/}
  timeout -k 10 300 $B --config $1 --set $2 > $O/$n.log 2>&1 || exit 1
  echo "$v $(grep -o '"value": [0-9.]*' $O/$n.log | head -1) $(grep -o '"raytrace": [0-9.]*' $O/$n.log | head -1)"
done
SNG_LIB_PATH=synerfgine_amd/_build_old/libsng_hip.so timeout -k 10 300 $B --config c3 > $O/c3_old.log 2>&1 && echo "old $(grep -o '"value": [0-9.]*' $O/c3_old.log | head -1)"
timeout -k 10 300 python3 -u tools/tile_cost.py --config c3 --bounds 501-560 --bounds 433-501 > $O/tile_cost.log 2>&1; grep '^{' $O/tile_cost.log
