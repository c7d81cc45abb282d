export TMPDIR=/tmp
for c in "concurrent_streams=0" "concurrent_streams=0,rt_spec=1" "rt_spec=0" "rt_spec=1"; do
  d=gpurun_out/bk_$(echo $c | tr ',=' '__')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 tools/band_kernels.py 491 551 $c 20 > $d.log 2>&1 || exit 1
  tail -1 $d.log
done
