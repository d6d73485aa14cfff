// path.hpp -- PGRT_MODE_PATH launchers (path.hip).
#pragma once

#include "trace.hpp"

namespace pgrt {

// Per-path state of one sample batch.  A path is named by its level-0 ray index (pid); queue
// entry i of bounce L carries pid_in[i] and its throughput thr_in[i] (bounce 0: pid = i, T = 1);
// acc[pid] is the path's radiance sum (k_finish reads it as a resolved level-0 colour).
struct PathState {
    const int* pid_in;
    const float4* thr_in;
    int* pid_out;
    float4* thr_out;
    float4* acc;
};

// one bounce's shading: misses add T * environment, dielectrics continue (reflect or refract),
// opaque hits emit hard shadow rays (sq from slot 0; contrib.w = the owning pid on a path's first
// shadow ray, -1 on the others) and a cosine-weighted continuation
void launch_path_shade(const SceneView& s, const FrameParams& fp, int width, const int4* tiles, int level, Queue q,
                       Queue next, const PathState& ps, ShadowQueue sq, FrameCounters* fc, int max_count, int expect,
                       hipStream_t stream);
// after the bounce's shadow rays are traced (sq.hit): the lit terms into acc, in light order
void launch_path_resolve(const SceneView& s, int level, ShadowQueue sq, const PathState& ps, const FrameCounters* fc,
                         int max_count, int expect, hipStream_t stream);

}  // namespace pgrt
