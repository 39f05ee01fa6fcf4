# A/B of the in-tree library against build/variants/lib_<v>.so at several dequeue chunks (dev
# tool); VARIANTS, CHUNKS and WORKLOADS select.  Solver GPU tests of the first variant first.
set -o pipefail
out=gpurun_out/abchunk; mkdir -p $out; log=$out/sweep.log; rm -f $log
first=${VARIANTS%% *}
SDK_LIB_PATH=$PWD/build/variants/lib_$first.so timeout -k 10 300 python -u -m pytest tests/test_gpu_solve.py tests/test_gpu_frontier.py \
  -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for wl in ${WORKLOADS:-solve17:1250000 solve17:10000000 solve30:1000000 minimal:1048576 hard:100000}; do
  w=${wl%%:*}; n=${wl##*:}
  for ch in ${CHUNKS:-0 8 4}; do
    for v in base $VARIANTS; do
      lib=""; [ $v != base ] && lib=$PWD/build/variants/lib_$v.so
      env ${lib:+SDK_LIB_PATH=$lib} timeout -k 10 120 python3 tools/solve_profile.py --solver quad --workload $w --n $n \
        --reps 5 --donate 0 --chunk $ch 2>&1 | sed "s/^/$v /" >> $log || exit 1
    done
  done
done
cat $log
