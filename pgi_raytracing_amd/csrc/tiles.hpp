// tiles.hpp -- how the image tiles of a distributed frame are dealt to ranks (host + device).
//
// Tiles are numbered row-major.  They are dealt in rounds of R = a + b * (world - 1) consecutive
// tiles: b sub-rounds of one tile per rank, rank 0 taking part in only the first a of them, so
// rank 0 renders a / b of another rank's share.  Rank 0 also unpacks every gathered frame into
// the framebuffer (≈ 10 µs per 1080p frame, ≈ 5 % of a C2 frame's render): with a < b the ranks
// finish together.  a == b is the plain round-robin deal (tile t -> rank t % world).
// The share is process-wide: PGRT_RANK0_SHARE="a/b" (1 <= a <= b <= 64), else a default by world
// size from the C2 measurements: 8/8 at 1-2 GPUs, 7/8 at 3-4, 6/8 at 5-7, 5/8 at 8+.
#pragma once

#include <cstdlib>
#include <cstdio>

namespace pgrt {

struct TileDeal {
    int world, a, b;
};

inline TileDeal tile_deal(int world) {
    static const int env_a = [] {
        const char* e = std::getenv("PGRT_RANK0_SHARE");
        int a = 0, b = 0;
        if (e && std::sscanf(e, "%d/%d", &a, &b) == 2 && a >= 1 && b >= a && b <= 64) return a * 100 + b;
        return 0;
    }();
    TileDeal d{world, 8, 8};
    if (env_a) {
        d.a = env_a / 100;
        d.b = env_a % 100;
    } else if (world >= 8) {
        // r1j emulated C2 ranks (tools/emulate_scaling.py, slowest rank ms/frame): 8 GPUs 5/8
        // 0.025 vs 4/8 0.027 (a round of 60 tiles = two rows of 30 puts every rank on fixed
        // columns, one of them over the canopy), 4 GPUs 7/8 0.054 vs 6/8 0.057, 2 GPUs 8/8
        // 0.100 vs 7/8 0.105
        d.a = 5;
    } else if (world >= 5) {
        d.a = 6;
    } else if (world >= 3) {
        d.a = 7;
    }
    if (world <= 1) d.a = d.b = 1;
    return d;
}

__host__ __device__ inline int deal_round(const TileDeal& d) { return d.a + d.b * (d.world - 1); }

// tile t -> (rank, local index j on that rank)
__host__ __device__ inline void deal_owner(const TileDeal& d, int t, int& rank, int& j) {
    if (d.world <= 1) {
        rank = 0;
        j = t;
        return;
    }
    const int R = deal_round(d), round = t / R, pos = t - round * R;
    if (pos < d.a * d.world) {
        const int sub = pos / d.world;
        rank = pos - sub * d.world;
        j = round * (rank == 0 ? d.a : d.b) + sub;
    } else {
        const int p2 = pos - d.a * d.world, sub = d.a + p2 / (d.world - 1);
        rank = 1 + p2 % (d.world - 1);
        j = round * d.b + sub;
    }
}

// (rank, local index j) -> tile t (may be >= the tile count: padding of the rank's list)
__host__ __device__ inline int deal_tile(const TileDeal& d, int rank, int j) {
    if (d.world <= 1) return j;
    const int R = deal_round(d);
    if (rank == 0) return (j / d.a) * R + (j % d.a) * d.world;
    const int round = j / d.b, sub = j % d.b;
    if (sub < d.a) return round * R + sub * d.world + rank;
    return round * R + d.a * d.world + (sub - d.a) * (d.world - 1) + (rank - 1);
}

// tiles of `rank` among `total`
inline int deal_count(const TileDeal& d, int total, int rank) {
    int lo = 0, hi = total + 1;  // deal_tile is increasing in j: the first j with tile >= total
    while (lo < hi) {
        const int mid = (lo + hi) / 2;
        if (deal_tile(d, rank, mid) < total) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// the longest rank list (the gather's per-rank block)
inline int deal_max_count(const TileDeal& d, int total) {
    int m = 0;
    for (int r = 0; r < d.world && r < 2; ++r) m = deal_count(d, total, r) > m ? deal_count(d, total, r) : m;
    return m;  // ranks >= 1 hold the same count or one less than rank 1
}

}  // namespace pgrt
