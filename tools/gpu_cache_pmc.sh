# L1 / L2 behaviour of the hot kernels: one PMC pass (2 TCC + 2 TCP counters) over the serialized bench
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc/CACHE -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --serial-streams > gpurun_out/pmc/CACHE.log 2>&1
rc=$?; echo "CACHE rc=$rc"; [ $rc -ne 0 ] && tail -20 gpurun_out/pmc/CACHE.log
exit $rc
