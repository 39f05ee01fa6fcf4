# rocprofv3 kernel traces of the 1M-board frontier build with expand_kernel and expand4_kernel (dev tool)
set -o pipefail
root=$(pwd); out=gpurun_out/frontier_prof; mkdir -p $out; export TMPDIR=/tmp
for s in halfwave quad; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d "$root/$out/$s" -o run --output-format csv -- \
     python3 "$root/tools/frontier_levels.py" $s > "$root/$out/$s.log" 2>&1) || { tail -5 $out/$s.log; exit 1; }
  cat $out/$s.log
  python3 tools/frontier_trace.py $(find $out/$s -name '*kernel_trace.csv') | tee $out/${s}_levels.txt
done
