// tiles.hpp -- how the image tiles of a distributed frame are dealt to ranks (host + device).
//
// Tiles are numbered row-major and dealt in rounds of R = a + b * (world - 1) consecutive tiles:
// rank 0 gets a tiles per round, every other rank b.  Inside a round, min(a, b) sub-rounds deal
// one tile to every rank in turn (tile -> rank tile % world), then either (b - a) sub-rounds deal
// one tile to each of ranks 1..world-1 (a < b) or the last (a - b) tiles go to rank 0 (a > b).
// a == b is the plain round-robin deal.  The interleaving spreads the glass-canopy hotspot over
// every rank.  Rank 0's share a/b trades its own rendering against the gather it receives and
// the unpack it runs: a < b when the unpack is the larger cost (C2 compute emulation, r1j), a > b
// when the xGMI ingress into rank 0 is (pgrt_tune_distribution measures it).
// Default by world size from the C2 emulation: 8/8 at 1-2 GPUs, 7/8 at 3-4,
// 6/8 at 5-7, 5/8 at 8+; PGRT_RANK0_SHARE="a/b" (1 <= a, b <= 64) overrides it process-wide.
#pragma once

#include <cstdlib>
#include <cstdio>

// host + device helpers; a host-only compile (tiles_abi.cpp under g++, make asan) sees plain inline
#if defined(__HIP__)
#define PGRT_TILE_HD __host__ __device__
#else
#define PGRT_TILE_HD
#endif

namespace pgrt {

struct TileDeal {
    int world, a, b;
};

inline TileDeal tile_deal(int world) {
    static const int env_a = [] {
        const char* e = std::getenv("PGRT_RANK0_SHARE");
        int a = 0, b = 0;
        if (e && std::sscanf(e, "%d/%d", &a, &b) == 2 && a >= 1 && a <= 64 && b >= 1 && b <= 64) return a * 100 + b;
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

// an explicit share (a, b >= 1); world 1 deals every tile to rank 0
inline TileDeal tile_deal(int world, int a, int b) {
    if (a <= 0 || b <= 0) return tile_deal(world);
    if (world <= 1) return TileDeal{world, 1, 1};
    return TileDeal{world, a, b};
}

PGRT_TILE_HD inline int deal_round(const TileDeal& d) { return d.a + d.b * (d.world - 1); }

// tile t -> (rank, local index j on that rank)
PGRT_TILE_HD inline void deal_owner(const TileDeal& d, int t, int& rank, int& j) {
    if (d.world <= 1) {
        rank = 0;
        j = t;
        return;
    }
    const int R = deal_round(d), round = t / R, pos = t - round * R;
    const int m = d.a < d.b ? d.a : d.b;
    if (pos < m * d.world) {
        const int sub = pos / d.world;
        rank = pos - sub * d.world;
        j = round * (rank == 0 ? d.a : d.b) + sub;
    } else if (d.a < d.b) {
        const int p2 = pos - m * d.world, sub = m + p2 / (d.world - 1);
        rank = 1 + p2 % (d.world - 1);
        j = round * d.b + sub;
    } else {
        rank = 0;
        j = round * d.a + m + (pos - m * d.world);
    }
}

// (rank, local index j) -> tile t (may be >= the tile count: padding of the rank's list)
PGRT_TILE_HD inline int deal_tile(const TileDeal& d, int rank, int j) {
    if (d.world <= 1) return j;
    const int R = deal_round(d);
    const int m = d.a < d.b ? d.a : d.b;
    if (rank == 0) {
        const int round = j / d.a, k = j % d.a;
        return k < m ? round * R + k * d.world : round * R + m * d.world + (k - m);
    }
    const int round = j / d.b, k = j % d.b;
    if (k < m) return round * R + k * d.world + rank;
    return round * R + m * d.world + (k - m) * (d.world - 1) + (rank - 1);
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

// the longest rank list
inline int deal_max_count(const TileDeal& d, int total) {
    int m = 0;
    for (int r = 0; r < d.world && r < 2; ++r) m = deal_count(d, total, r) > m ? deal_count(d, total, r) : m;
    return m;  // ranks >= 1 hold the same count or one less than rank 1
}

// exclusive prefix of the rank lists: the rank-major position of rank r's first tile
inline long long deal_offset(const TileDeal& d, int total, int rank) {
    long long o = 0;
    for (int r = 0; r < rank; ++r) o += deal_count(d, total, r);
    return o;
}

// ---- the tail of a rank's distributed send (distributed.cpp collect_frame) ----
// Two words after the rank's tiles: the flag (0 the frame is good, 1 its queues overflowed -- it
// re-renders and sends again, 2 it gave up: "poison"), then the frame's sequence number (the
// rank's count of distributed frames; 0 = nothing received from that rank in this gather).
enum { kTailOk = 0, kTailOverflow = 1, kTailPoison = 2 };
PGRT_TILE_HD inline int gather_tail_flag(bool overflow, bool poison) {
    return poison ? kTailPoison : (overflow ? kTailOverflow : kTailOk);
}
// Rank 0's reading of the peers' tails of one gather: 0 and regather[r] = 1 for every rank whose
// tiles must be received again; or -1 with *bad = the first rank that sent another frame's tiles
// (the ranks do not submit / wait in the same order); or -2 with *bad = a rank that gave up.
inline int gather_tail_verdict(const int* flags, const unsigned* seqs, int world, unsigned expect, int* regather,
                               int* bad) {
    for (int r = 0; r < world; ++r) regather[r] = 0;
    for (int r = 1; r < world; ++r) {
        if (seqs[r] == 0) continue;  // not received in this gather (a re-gather of other ranks)
        if (seqs[r] != expect) {
            *bad = r;
            return -1;
        }
        if (flags[r] == kTailPoison) {
            *bad = r;
            return -2;
        }
        regather[r] = flags[r] != kTailOk;
    }
    return 0;
}

}  // namespace pgrt
