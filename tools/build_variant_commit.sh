# Build libsudoku_hip.so of another commit into build/variants/lib_<name>.so (dev tool, A/B timing)
# usage: tools/build_variant_commit.sh <name> <commit> [extra hipcc flags...]
set -e
name=$1; commit=$2; shift 2
tmp=build/variants/git_$name; rm -rf $tmp; mkdir -p $tmp
git archive $commit distributed_sudoku_solver_amd/csrc include | tar -x -C $tmp
S=$tmp/distributed_sudoku_solver_amd/csrc
out=build/variants/$name; rm -rf $out; mkdir -p $out
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-result $*"
$H -c -o $out/a.o $S/sudoku_hip.hip &
$H -mllvm -simplifycfg-sink-common=false -c -o $out/b.o $S/solve2_launch.hip &
$H -mllvm -simplifycfg-sink-common=false -c -o $out/c.o $S/solve4_launch.hip &
[ -f $S/prop32_launch.hip ] && $H -fno-slp-vectorize -fno-vectorize -c -o $out/d.o $S/prop32_launch.hip &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/variants/lib_$name.so $out/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
