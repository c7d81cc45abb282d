set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
for v in 32 16 24 48 64 32; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-sweep --config c3 --set rt_reserved_cus=$v > $O/c3_$v.log 2>&1 || exit 1
  echo "reserved $v $(grep -o '"value": [0-9.]*' $O/c3_$v.log | head -1) $(grep -o '"raytrace": [0-9.]*' $O/c3_$v.log | head -1) $(grep -o '"nerf": [0-9.]*' $O/c3_$v.log | head -1)"
done
