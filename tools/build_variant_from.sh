# Build a variant whose solve4/solve2 headers come from another directory (dev tool, A/B timing):
# usage: tools/build_variant_from.sh <name> <dir with solve4_kernel.h [solve2_kernel.h]> [extra hipcc flags...]
set -e
name=$1; src=$2; shift 2
tmp=build/variants/src_$name; rm -rf $tmp; mkdir -p $tmp
cp distributed_sudoku_solver_amd/csrc/*.h distributed_sudoku_solver_amd/csrc/*.hip $tmp/
mkdir -p build/include && cp include/sudoku_hip.h build/include/
cp $src/*.h $tmp/
out=build/variants/$name; mkdir -p $out
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-result -I$PWD/include $*"
$H -c -o $out/a.o $tmp/sudoku_hip.hip &
$H -mllvm -simplifycfg-sink-common=false -c -o $out/b.o $tmp/solve2_launch.hip &
$H -mllvm -simplifycfg-sink-common=false -c -o $out/c.o $tmp/solve4_launch.hip &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/variants/lib_$name.so $out/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
