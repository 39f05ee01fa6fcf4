// frontier_args.h -- the frontier build's control block and expansion arguments, shared by
// frontier_kernel.h (sudoku_hip.hip) and expand4_kernel.h (solve4_launch.hip).
#pragma once
#include <cstdint>

namespace sdk {

// device-side control block of one frontier build
struct FrontierCtl {
    unsigned long long m;        // boards in the current frontier
    unsigned long long leaves;   // completions met while expanding (count mode), accepted levels only
    unsigned long long lvl_leaves;  // completions met by the level being expanded (folded into
                                    // `leaves` by frontier_end_kernel only if the level is accepted)
    unsigned long long open;     // boards that branched in the current level
    unsigned long long total;    // children of the current level (scan)
    unsigned int level;          // completed levels: the frontier is in buffer (level & 1)
    unsigned int done;           // 1 = expansion finished
    unsigned int next;           // expand_kernel dequeue counter
    unsigned int pad;
};

constexpr int kScanTile = 4096;   // entries per scan tile (1024 threads x 4)

struct ExpandArgs {
    const uint8_t* in;
    FrontierCtl* ctl;
    uint8_t* prop;            // [m][81] propagated board (singles as givens)
    uint8_t* bcell;           // [m] branch cell
    uint16_t* bmask;          // [m] branch candidates (bit d-1 = digit d)
    uint32_t* nchild;         // [m]
    int order;
    const uint16_t* mask;      // nullable, level 0 only: first-cell digit mask of every seed board
    int keep_leaves;           // first-solution mode (see header)
};

constexpr uint16_t kKeepBoard = 0x8000;   // bmask flag: emit the propagated board itself

}  // namespace sdk
