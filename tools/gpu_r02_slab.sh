set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r02_slab; mkdir -p $O
timeout -k 10 300 python -u bench.py --workload nodes512 --steps 10 --warmup 2 --no-cpu-baseline > $O/tensor.log 2>&1 || exit 1
tail -1 $O/tensor.log | cut -c1-300
timeout -k 10 300 python -u bench.py --workload nodes512 --steps 10 --warmup 2 --no-cpu-baseline --alloc slab > $O/slab.log 2>&1 || exit 1
tail -1 $O/slab.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -T -d $R/$O/trace -o run --output-format csv -- python3 $R/bench.py --workload nodes512 --steps 3 --warmup 1 --no-cpu-baseline --alloc slab > $R/$O/trace.log 2>&1 || exit 1
echo done
