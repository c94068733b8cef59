// kle_brick.hpp -- the brick decomposition of the box symmetric SpMV
// (kle_brick.hip: kernels and device set-up; kle_brick_plan.cpp: the host
// planner, also reachable on a CPU through kle_brick_plan_box).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace kle {

// per brick (device, 80 B): the bounding box of its rows in owned-lattice
// coordinates (a box, or a ragged band piece whose first and last x planes /
// y lines are partial), its row count, the region (bounding box of its rows'
// upper triangles; z in owned coordinates), its first row descriptor, the
// bound exponent of its fixed-point sums, where its values and its region
// sums live
struct BrickDesc {
    int x0, y0, z0, nx, ny, nz;
    int ox, oy, oz, RX, RY, RZ;
    int rstart, eb, nr, pad_;
    long long vbase, wsoff;
};
static_assert(sizeof(BrickDesc) == 80, "BrickDesc layout");

// a row descriptor: word 0 the packed row box (dbx, dby, dbz, bnx, bny, bnz:
// 4 bits each) + the low byte of its region index; word 1 its value offset
// / 16 doubles (23 bits), BRICK_ROW_NULL (a unit's absent second row) and the
// high byte of the region index.  Rows come in units of two (kle_brick_plan.cpp).
constexpr int BRICK_ROW_NULL = 1 << 23;
inline bool brick_row_null(const int *rowd, int64_t r) { return (rowd[2 * r + 1] & BRICK_ROW_NULL) != 0; }
// a row descriptor's region index (the low and high bytes of its two words)
inline int brick_row_ir(const int *rowd, int64_t r)
{
    return ((rowd[2 * r] >> 24) & 255) | (((rowd[2 * r + 1] >> 24) & 255) << 8);
}
// the owned-lattice node of region index ir of brick D
inline int64_t brick_ir_node(const BrickDesc &D, int ir, int64_t Lx, int64_t Ly)
{
    const int rxy = D.RX * D.RY, rz = ir / rxy, rem = ir - rz * rxy, ry = rem / D.RX, rx = rem - ry * D.RX;
    return (D.ox + rx) + Lx * ((D.oy + ry) + Ly * (int64_t)(D.oz + rz));
}

constexpr int BRICK_MAX_ROUNDS = 8;        // bricks per CU the planner goes up to when fewer do not fit the LDS
constexpr int BRICK_WV = 16;            // waves per brick workgroup (one workgroup per CU)
constexpr size_t BRICK_LDS_CAP = 163840;  // LDS per CU
constexpr size_t BRICK_LDS_MIN = 82 * 1024;  // above half the CU's LDS: never two bricks on one CU

// dynamic LDS of a brick: x [3][RN] | sums [3][RN + 64] (64 dummy slots per
// component take the adds of masked lanes) | wave maxima, row counter

struct BrickPlan {
    std::vector<BrickDesc> bricks;  // the bricks (tail tiles last), in launch order
    std::vector<int> rowd;      // 2 ints per row, brick order
    std::vector<int64_t> svb;   // per row (natural index): first double of its values, brick layout
    int64_t ws_doubles = 0, ws_entries = 0;
    size_t lds = 0;
    double model_us = 0.0;  // the planner's time model of the product (us)
    int singles = 0;        // (in) rows of one stored block out of the bricks, to the gather (spmv_brick_singles)
    int pair = 0;           // (in) units of two rows sharing their tails' item (spmv_brick_pair)
    std::vector<int64_t> srows;  // (out) those rows, ascending; their values (9 doubles each) after the bricks'
};

// the plan's tables checked against every address the brick kernel forms
// from them (kle_brick_plan.cpp); nullptr: consistent, else what is wrong
const char *brick_validate(const BrickPlan &bp, int64_t Lx, int64_t Ly, int64_t Lz, int64_t nvals, int64_t lds_cap);
// the LDS a brick of RN region nodes needs (x, the transposed sums and their
// dummy slots, wave maxima, the row counter)
inline size_t brick_lds(int RN) { return (size_t)(3 * RN + 3 * (RN + 64)) * 8 + 512; }
// an unstructured (graph) brick: rows [r0, r0 + nr), its dictionary of U
// entries from dict[d0] (its rows first), values from sval[vbase], 2-byte
// positions from slid[sbase], sums to ws[wsoff] ([entry][3]); eb its bound
// (kle_gbrick.hip)
struct GBrickDesc {
    int r0, nr, U, eb;
    long long d0, vbase, sbase, wsoff;
};
// dictionary entries a graph brick may hold (brick_lds <= BRICK_LDS_CAP)
constexpr int GB_UCAP = (int)((BRICK_LDS_CAP - 2048) / 48);

// bricks for the owned Lx x Ly x Lz lattice of a rank (rows x-fastest; per
// row its block count and packed box, kle_sym.hip srow; hp upper ghost
// planes, z slabs at N > 1) on ncu CUs: at
// most `rounds` bricks per CU, or at most nfix bricks (> 0); fs: forced
// split counts (0: planned).  "" or why not.
std::string brick_plan(int Lx, int Ly, int Lz, int hp, int ncu, int nfix, int rounds, int fs, const std::vector<int> &cnt,
                       const std::vector<int> &srow, int P, BrickPlan &bp);

}  // namespace kle
