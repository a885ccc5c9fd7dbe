// le_bricks.h -- brick numbering of the key-cell grid (host + device).
//
// Brick coordinates bc[d] in [0, nb[d]) (nb a multiple of TILE=4).  Brick id =
// tile * 4^NDIM + morton(bc % 4), tile = linear index of bc / 4 (x fastest).
// Consecutive ids stay inside a 32^3-cell tile, so the bricks one XCD works on
// at a time are spatially compact (their halos are shared through L2/MALL), and
// an aligned 2x2(x2) group of bricks -- a spread super-brick -- is 2^NDIM
// consecutive ids starting at a multiple of 2^NDIM.
#pragma once
#include <hip/hip_runtime.h>

#include "le_internal.h"

namespace ibtk_le {

template <int NDIM> struct BrickT {
    static constexpr int B = NDIM == 3 ? BRICK3 : BRICK2;  // cells per brick edge
    static constexpr int BV = NDIM == 3 ? B * B * B : B * B;
    static constexpr int SHIFT = NDIM == 3 ? 9 : 8;         // log2(BV)
    static constexpr int TV = NDIM == 3 ? 64 : 16;          // bricks per tile
    static constexpr int TSHIFT = NDIM == 3 ? 6 : 4;
    static constexpr int SB = 2 * B;                        // super-brick edge (cells)
    static constexpr int SBV = NDIM == 3 ? SB * SB * SB : SB * SB;
    static constexpr int GROUP = NDIM == 3 ? 8 : 4;         // bricks per super-brick
};

// 2-bit-per-dim Morton code of a brick inside its tile (coords 0..3)
template <int NDIM> __host__ __device__ __forceinline__ int morton_local(int x, int y, int z) {
    if (NDIM == 3)
        return (x & 1) | ((y & 1) << 1) | ((z & 1) << 2) | ((x & 2) << 2) | ((y & 2) << 3) | ((z & 2) << 4);
    return (x & 1) | ((y & 1) << 1) | ((x & 2) << 1) | ((y & 2) << 2);
}

template <int NDIM> __host__ __device__ __forceinline__ void morton_decode(int m, int* c) {
    if (NDIM == 3) {
        c[0] = (m & 1) | ((m >> 2) & 2);
        c[1] = ((m >> 1) & 1) | ((m >> 3) & 2);
        c[2] = ((m >> 2) & 1) | ((m >> 4) & 2);
    } else {
        c[0] = (m & 1) | ((m >> 1) & 2);
        c[1] = ((m >> 1) & 1) | ((m >> 2) & 2);
        c[2] = 0;
    }
}

template <int NDIM> __host__ __device__ __forceinline__ int brick_id(const BinGeom& bg, const int* bc) {
    int t = 0;
    for (int d = NDIM - 1; d >= 0; --d) t = t * bg.nt[d] + (bc[d] >> 2);
    return (t << BrickT<NDIM>::TSHIFT) | morton_local<NDIM>(bc[0] & 3, bc[1] & 3, NDIM == 3 ? (bc[2] & 3) : 0);
}

template <int NDIM> __host__ __device__ __forceinline__ void brick_coords(const BinGeom& bg, int b, int* bc) {
    int t = b >> BrickT<NDIM>::TSHIFT;
    int l[3];
    morton_decode<NDIM>(b & (BrickT<NDIM>::TV - 1), l);
    for (int d = 0; d < NDIM; ++d) {
        bc[d] = (t % bg.nt[d]) * 4 + l[d];
        t /= bg.nt[d];
    }
    if (NDIM == 2) bc[2] = 0;
}

// blocks are dealt round-robin over the 8 XCDs (blockIdx % 8 labels an XCD):
// give XCD x the contiguous item range [x*G/8, (x+1)*G/8) of each round so the
// items an XCD runs together are neighbours.  Speed only, never correctness.
__device__ __forceinline__ int xcd_item(int round_base, int G, int wg) {
    if (G & 7) return round_base + wg;
    const int per = G >> 3;
    return round_base + (wg & 7) * per + (wg >> 3);
}

}  // namespace ibtk_le
