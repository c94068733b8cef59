// kle_sym_dev.hpp -- device helpers shared by the symmetric-storage SpMV
// kernels (kle_sym.hip: tile and graph kernels; kle_brick.hip: brick kernel):
// DPP wave sums, exact int64 fixed-point conversions, the value-load asm with
// explicit vmcnt waits, block-position divisions.
#pragma once
#include "kle_internal.hpp"

namespace kle {

// Wave sums through DPP row moves (VALU only; __shfl_xor is a ds_bpermute per
// 32-bit half, i.e. 12 LDS instructions per double): quad swaps, half-row
// and row mirrors, then row_bcast15 / row_bcast31 carry the row sums into
// lane 63, which every lane reads back.  Three sums at once, their steps
// interleaved (no hazard nops between a step's add and the next step's DPP
// read); the full-row steps use the source as the unused "old" operand
// (every lane is written), only the row broadcasts need zeros.
template <int ctrl, int row_mask>
__device__ __forceinline__ void dpp3(double &a, double &b, double &c)
{
    constexpr bool all = row_mask == 0xF;
    const int al = __double2loint(a), ah = __double2hiint(a), bl = __double2loint(b), bh = __double2hiint(b);
    const int cl = __double2loint(c), ch = __double2hiint(c);
    const int a2 = __builtin_amdgcn_update_dpp(all ? al : 0, al, ctrl, row_mask, 0xF, false);
    const int a3 = __builtin_amdgcn_update_dpp(all ? ah : 0, ah, ctrl, row_mask, 0xF, false);
    const int b2 = __builtin_amdgcn_update_dpp(all ? bl : 0, bl, ctrl, row_mask, 0xF, false);
    const int b3 = __builtin_amdgcn_update_dpp(all ? bh : 0, bh, ctrl, row_mask, 0xF, false);
    const int c2 = __builtin_amdgcn_update_dpp(all ? cl : 0, cl, ctrl, row_mask, 0xF, false);
    const int c3 = __builtin_amdgcn_update_dpp(all ? ch : 0, ch, ctrl, row_mask, 0xF, false);
    a += __hiloint2double(a3, a2);
    b += __hiloint2double(b3, b2);
    c += __hiloint2double(c3, c2);
}

__device__ __forceinline__ void wsum3_dpp(double &a, double &b, double &c)
{
    dpp3<0xB1, 0xF>(a, b, c);   // quad_perm [1,0,3,2]
    dpp3<0x4E, 0xF>(a, b, c);   // quad_perm [2,3,0,1]
    dpp3<0x141, 0xF>(a, b, c);  // row_half_mirror
    dpp3<0x140, 0xF>(a, b, c);  // row_mirror
    dpp3<0x142, 0xA>(a, b, c);  // row_bcast15 into rows 1, 3
    dpp3<0x143, 0xC>(a, b, c);  // row_bcast31 into rows 2, 3
    a = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(a), 63), __builtin_amdgcn_readlane(__double2loint(a), 63));
    b = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(b), 63), __builtin_amdgcn_readlane(__double2loint(b), 63));
    c = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(c), 63), __builtin_amdgcn_readlane(__double2loint(c), 63));
}

// q = n / d for 0 <= n < 2^20, d >= 1 (block position in its row box)
__device__ __forceinline__ int sym_div(int n, int d, float inv)
{
    int q = (int)((float)n * inv);
    q += (q + 1) * d <= n;
    q -= q * d > n;
    return q;
}

__device__ __forceinline__ double uni_d(double v)
{
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
    const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}


__device__ __forceinline__ unsigned long long fx_of(double c, double S)
{
    const double v = __builtin_rint(c * S);           // |v| <= 2^61: an integer
    const double hi = __builtin_floor(v * 0x1p-32);  // exact
    const double lo = __builtin_fma(hi, -0x1p32, v);  // exact, in [0, 2^32)
    return ((unsigned long long)(unsigned)(int)hi << 32) + (unsigned long long)(unsigned)lo;
}

__device__ __forceinline__ double fx_to_d(unsigned long long u)
{
    return (double)(int)((long long)u >> 32) * 0x1p32 + (double)(unsigned)(u & 0xffffffffull);
}

// Value loads of one item of k_nb_spmv_sym_xl, issued in inline asm so the
// compiler's wait bookkeeping cannot drain them: it saw the next item's loads
// as hazards on registers of the current one and put s_waitcnt vmcnt(0) in
// front of them at every second item.  The wait for an item (vmcnt(9): the
// next item's 9 loads stay in flight) names its 9 registers as read-write
// operands, so nothing reads them before the data has landed.
__device__ __forceinline__ void sym_ld9(double *v, const double *base, const unsigned *o)
{
    asm volatile(
        "s_nop 4\n\t"
        "global_load_dwordx2 %0, %9, %18 nt\n\t"
        "global_load_dwordx2 %1, %10, %18 nt\n\t"
        "global_load_dwordx2 %2, %11, %18 nt\n\t"
        "global_load_dwordx2 %3, %12, %18 nt\n\t"
        "global_load_dwordx2 %4, %13, %18 nt\n\t"
        "global_load_dwordx2 %5, %14, %18 nt\n\t"
        "global_load_dwordx2 %6, %15, %18 nt\n\t"
        "global_load_dwordx2 %7, %16, %18 nt\n\t"
        "global_load_dwordx2 %8, %17, %18 nt"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]),
          "=&v"(v[8])
        : "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "v"(o[4]), "v"(o[5]), "v"(o[6]), "v"(o[7]), "v"(o[8]),
          "s"(base)
        : "memory");
}

template <int N>
__device__ __forceinline__ void sym_wait9(double *v)
{
    asm volatile("s_waitcnt vmcnt(%9)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
                   "+v"(v[8])
                 : "i"(N));
}

// One load of x for a brick's region fill (SGPR base + 32-bit byte offset),
// in inline asm like the value loads: issued before the first items' value loads, it is waited for with
// an explicit vmcnt that leaves those in flight (a compiler load would be
// waited for with vmcnt(0) once the asm loads follow it).
__device__ __forceinline__ void ld_x1(double &v, const double *base, unsigned byte_off)
{
    asm volatile("global_load_dwordx2 %0, %1, %2" : "=&v"(v) : "v"(byte_off), "s"(base) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_x12(double *v)
{
    asm volatile("s_waitcnt vmcnt(%12)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
                   "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11])
                 : "i"(N));
}

}  // namespace kle
