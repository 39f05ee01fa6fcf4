# Build the current csrc tree into build/variants/lib_<name>.so (dev tool, for tools/q2.sh VARIANTS=...)
# usage: tools/build_variant.sh <name> [extra hipcc flags...]
set -e
name=$1; shift
out=build/variants/$name; mkdir -p $out
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-result $*"
S=distributed_sudoku_solver_amd/csrc
$H -c -o $out/a.o $S/sudoku_hip.hip &
$H -mllvm -simplifycfg-sink-common=false -c -o $out/b.o $S/solve2_launch.hip &
$H -mllvm -simplifycfg-sink-common=false -c -o $out/c.o $S/solve4_launch.hip &
[ -f $S/prop32_launch.hip ] && $H -fno-slp-vectorize -fno-vectorize -c -o $out/d.o $S/prop32_launch.hip &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/variants/lib_$name.so $out/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
