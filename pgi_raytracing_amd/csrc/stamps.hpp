// stamps.hpp -- device-stamped launch timeline (pgrt_timeline_enable / pgrt_timeline_read).
//
// Every frame-path kernel can stamp its own span on the device clock, without rocprof or HIP
// events: each wave writes {first s_memrealtime after entry, last one before exit} (100 MHz
// ticks, one 16-B store per wave) into a slot range its launcher reserved; the host reduces a
// launch's range to (min start, max end).  Off (the default), the launchers pass no slot range
// and the kernels skip the stamps on a uniform kernel-argument branch.  The reference's frame loop
// (SimpleGuiDX11::Producer, APP/simpleguidx11.cpp:95-124) has no timing at all; this is the
// measurement the latency work is decided on.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

namespace pgrt {

// kernel kinds of a timeline record (pgrt.h PGRT_TL_*)
enum StampKind : int {
    kStampRaygen = 0,
    kStampTracePkt,
    kStampTrace,
    kStampTrace8g,
    kStampTraceResume,
    kStampTraceShadow,
    kStampShade,
    kStampCombine,
    kStampFinish,
    kStampExport,
    kStampUnpack,
    kStampPathShade,
    kStampPathResolve,
    kStampSubtree,
    kStampExportTiles,
    kStampKinds
};

// one launch's reserved stamp range (host side)
struct StampLaunch {
    int kind, level, slot;
    long long offset;  // first wave's slot (16 B each) in the frame set's stamp buffer
    int waves;
};

// The stamp log of the frame set being enqueued (set by enqueue_frame for the launches of one
// pipeline slot); launchers take their slot range from it.  NULL: no timeline.
struct StampLog {
    unsigned long long* dev = nullptr;  // 2 words per wave: start, end
    long long cap = 0;                  // waves the buffer holds
    long long used = 0;
    int slot = 0;
    std::vector<StampLaunch>* launches = nullptr;
    bool overflow = false;
};
void set_stamp_log(StampLog* log);
StampLog* stamp_log();

// the slot range of a launch of grid x block threads (1-D block, waves of 64): NULL without a log
// or when the buffer is full (the launch is then not recorded)
inline unsigned long long* stamp_next(int kind, int level, long long grid, int block) {
    StampLog* l = stamp_log();
    if (!l || !l->dev) return nullptr;
    const long long waves = grid * ((block + 63) / 64);
    if (l->used + waves > l->cap) {
        l->overflow = true;
        return nullptr;
    }
    unsigned long long* p = l->dev + 2 * l->used;
    l->launches->push_back(StampLaunch{kind, level, l->slot, l->used, (int)waves});
    l->used += waves;
    return p;
}

// device side: the wave's stamp pair.  PGRT_STAMP_BEGIN at kernel entry, PGRT_STAMP_END after the
// kernel body has returned (every lane of the wave active again: bodies with early returns are
// separate inline functions)
#ifndef PGRT_STAMPS
#define PGRT_STAMPS 1
#endif
#if !PGRT_STAMPS  // A/B builds: no stamp code in the kernels at all
#define PGRT_STAMP_BEGIN(ptr) (void)(ptr)
#define PGRT_STAMP_END(ptr) (void)(ptr)
#else
// The entry stamp is a non-volatile asm: the s_memrealtime builtin is a memory side effect to
// LLVM, and one at kernel entry marks every later load as possibly clobbered -- uniform loads of
// read-only data (queue counts, packet-traversal nodes) then compile to vector loads instead of
// scalar ones, 15-30% off every kernel even with the stamps off.  The asm is convergent (device
// code), so it is neither sunk nor merged into the exit stamp (a different instruction).
__device__ __forceinline__ unsigned long long stamp_clock_entry() {
    unsigned long long t;
    asm("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    return t;
}
#define PGRT_STAMP_BEGIN(ptr) const unsigned long long pgrt_stamp_t0_ = (ptr) ? stamp_clock_entry() : 0ull
#define PGRT_STAMP_END(ptr)                                                                              \
    do {                                                                                                 \
        if (ptr) {                                                                                       \
            const unsigned long long t1_ = wall_clock64();                                               \
            if (__lane_id() == 0) {                                                                      \
                const long long w_ = ((long long)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + \
                                     (threadIdx.x >> 6);                                                 \
                reinterpret_cast<ulonglong2*>(ptr)[w_] = make_ulonglong2(pgrt_stamp_t0_, t1_);           \
            }                                                                                            \
        }                                                                                                \
    } while (0)
#endif

}  // namespace pgrt
