// tiles_abi.cpp -- the tile deal of distributed frames as host-only C ABI entry points
// (pgrt_tile_*, pgrt_unpack_tiles_host*; tiles.hpp): no HIP, so the sanitizer build (make asan)
// compiles it with g++ beside the OBJ loader.
#include <algorithm>
#include <cstring>

#include "pgrt.h"
#include "tiles.hpp"

using namespace pgrt;

extern "C" {

int pgrt_tile_count_ex(int width, int height, int tile_size, int rank, int world, int a, int b) {
    if (width <= 0 || height <= 0 || tile_size <= 0 || world <= 0 || rank < 0 || rank >= world || a < 0 || b < 0 ||
        a > 64 || b > 64)
        return PGRT_ERR_INVALID_ARGUMENT;
    const long long total = (long long)((width + tile_size - 1) / tile_size) * ((height + tile_size - 1) / tile_size);
    return deal_count(tile_deal(world, a, b), (int)total, rank);
}

int pgrt_tile_index_ex(int width, int height, int tile_size, int rank, int world, int a, int b, int j) {
    if (width <= 0 || height <= 0 || tile_size <= 0 || world <= 0 || rank < 0 || rank >= world || j < 0 || a < 0 ||
        b < 0 || a > 64 || b > 64)
        return PGRT_ERR_INVALID_ARGUMENT;
    const int total = ((width + tile_size - 1) / tile_size) * ((height + tile_size - 1) / tile_size);
    const int t = deal_tile(tile_deal(world, a, b), rank, j);
    return t < total ? t : PGRT_ERR_INVALID_ARGUMENT;
}

int pgrt_tile_count(int width, int height, int tile_size, int rank, int world) {
    return pgrt_tile_count_ex(width, height, tile_size, rank, world, 0, 0);
}

int pgrt_tile_index(int width, int height, int tile_size, int rank, int world, int j) {
    return pgrt_tile_index_ex(width, height, tile_size, rank, world, 0, 0, j);
}

int pgrt_gather_tail(int overflow, int poison, unsigned seq, int tail[2]) {
    if (!tail || seq == 0) return PGRT_ERR_INVALID_ARGUMENT;
    tail[0] = gather_tail_flag(overflow != 0, poison != 0);
    tail[1] = (int)seq;
    return PGRT_OK;
}

int pgrt_gather_tail_verdict(const int* flags, const unsigned* seqs, int world, unsigned expect_seq, int* regather,
                             int* bad_rank) {
    if (!flags || !seqs || !regather || world < 1 || world > 64 || expect_seq == 0) return PGRT_ERR_INVALID_ARGUMENT;
    int bad = -1;
    const int v = gather_tail_verdict(flags, seqs, world, expect_seq, regather, &bad);
    if (bad_rank) *bad_rank = bad;
    return v == 0 ? PGRT_OK : (v == -1 ? PGRT_ERR_RCCL : PGRT_ERR_OUT_OF_MEMORY);
}

int pgrt_tile_share(int world, int* a, int* b) {
    if (world <= 0 || !a || !b) return PGRT_ERR_INVALID_ARGUMENT;
    const TileDeal d = tile_deal(world);
    *a = d.a;
    *b = d.b;
    return PGRT_OK;
}

int pgrt_tile_rect(int width, int height, int tile_size, int t, int rect[4]) {
    if (width <= 0 || height <= 0 || tile_size <= 0 || !rect) return PGRT_ERR_INVALID_ARGUMENT;
    const int tx = (width + tile_size - 1) / tile_size, ty = (height + tile_size - 1) / tile_size;
    if (t < 0 || t >= tx * ty) return PGRT_ERR_INVALID_ARGUMENT;
    rect[0] = (t % tx) * tile_size;
    rect[1] = (t / tx) * tile_size;
    rect[2] = std::min(tile_size, width - rect[0]);
    rect[3] = std::min(tile_size, height - rect[1]);
    return PGRT_OK;
}

int pgrt_unpack_tiles_host(int width, int height, int tile_size, int world, const float* g, float* rgba) {
    return pgrt_unpack_tiles_host_ex(width, height, tile_size, world, 0, 0, g, rgba);
}

int pgrt_unpack_tiles_host_ex(int width, int height, int tile_size, int world, int a, int b, const float* g,
                              float* rgba) {
    if (width <= 0 || height <= 0 || tile_size <= 0 || world <= 0 || !g || !rgba || a < 0 || b < 0 || a > 64 || b > 64)
        return PGRT_ERR_INVALID_ARGUMENT;
    const int tx = (width + tile_size - 1) / tile_size, ty = (height + tile_size - 1) / tile_size;
    const int total = tx * ty;
    const TileDeal d = tile_deal(world, a, b);
    const size_t tile_floats = (size_t)tile_size * tile_size * 4;
    size_t slot = 0;  // rank-major, each rank's tiles in its local order, no padding
    for (int r = 0; r < world; ++r)
        for (int j = 0; j < deal_count(d, total, r); ++j, ++slot) {
            const int t = deal_tile(d, r, j);
            const float* src = g + slot * tile_floats;
            const int x0 = (t % tx) * tile_size, y0 = (t / tx) * tile_size;
            for (int y = 0; y < tile_size && y0 + y < height; ++y)
                for (int x = 0; x < tile_size && x0 + x < width; ++x)
                    std::memcpy(rgba + ((size_t)(y0 + y) * width + (x0 + x)) * 4,
                                src + ((size_t)y * tile_size + x) * 4, 4 * sizeof(float));
        }
    return PGRT_OK;
}

}  // extern "C"
