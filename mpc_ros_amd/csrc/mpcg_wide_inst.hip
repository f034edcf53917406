// mpc_ros_amd/csrc/mpcg_wide_inst.hip -- the solver kernel instances, one group per
// translation unit: build.py compiles this file once per MPCG_INST value (0..11, in
// parallel) and links the objects into libmpcg.so.  The groups are listed with their
// instances in mpcg_wide_kern.h (MPCG_WIDE_SOLVE_INSTANCES / MPCG_WIDE_RESUME_INSTANCES).
#include "mpcg_wide_kern.h"

#ifndef MPCG_INST
#error "compile with -DMPCG_INST=<group>"
#endif

namespace mpcg {

#define MPCG_DEF_SOLVE(g, M, S, T, NB, D, W)                                                  \
    template <>                                                                               \
    const void* solve_kernel_fn<M, S, T, NB, D, W>() {                                       \
        return (const void*)k_solve_wide<M, S, T, NB, D, W>;                                  \
    }
#define MPCG_DEF_WARM(g, M, S, T, NB, D, W)                                                   \
    template <>                                                                               \
    const void* warm_kernel_fn<M, S, T, NB, D, W>() {                                        \
        return (const void*)k_warm_wide<M, S, T, NB, D, W>;                                   \
    }
#define MPCG_DEF_RESUME(g, M, S, T, NB)                                                       \
    template <>                                                                               \
    const void* resume_kernel_fn<M, S, T, NB>() {                                            \
        return (const void*)k_resume_wide<M, S, T, NB>;                                       \
    }
// (MPCG_SEL_<g>: the instance's definition if g is this unit's group, nothing otherwise)
#define MPCG_SEL_SOLVE(g, M, S, T, NB, D, W) MPCG_SEL_##g(MPCG_DEF_SOLVE(g, M, S, T, NB, D, W))
#define MPCG_SEL_RESUME(g, M, S, T, NB) MPCG_SEL_##g(MPCG_DEF_RESUME(g, M, S, T, NB))
#define MPCG_SEL_WARM(g, M, S, T, NB, D, W) MPCG_SEL_##g(MPCG_DEF_WARM(g, M, S, T, NB, D, W))
#if MPCG_INST == 0
#define MPCG_SEL_0(x) x
#else
#define MPCG_SEL_0(x)
#endif
#if MPCG_INST == 1
#define MPCG_SEL_1(x) x
#else
#define MPCG_SEL_1(x)
#endif
#if MPCG_INST == 2
#define MPCG_SEL_2(x) x
#else
#define MPCG_SEL_2(x)
#endif
#if MPCG_INST == 3
#define MPCG_SEL_3(x) x
#else
#define MPCG_SEL_3(x)
#endif
#if MPCG_INST == 4
#define MPCG_SEL_4(x) x
#else
#define MPCG_SEL_4(x)
#endif
#if MPCG_INST == 5
#define MPCG_SEL_5(x) x
#else
#define MPCG_SEL_5(x)
#endif
#if MPCG_INST == 6
#define MPCG_SEL_6(x) x
#else
#define MPCG_SEL_6(x)
#endif
#if MPCG_INST == 7
#define MPCG_SEL_7(x) x
#else
#define MPCG_SEL_7(x)
#endif
#if MPCG_INST == 8
#define MPCG_SEL_8(x) x
#else
#define MPCG_SEL_8(x)
#endif
#if MPCG_INST == 9
#define MPCG_SEL_9(x) x
#else
#define MPCG_SEL_9(x)
#endif
#if MPCG_INST == 10
#define MPCG_SEL_10(x) x
#else
#define MPCG_SEL_10(x)
#endif
#if MPCG_INST == 11
#define MPCG_SEL_11(x) x
#else
#define MPCG_SEL_11(x)
#endif
MPCG_WIDE_SOLVE_INSTANCES(MPCG_SEL_SOLVE)
MPCG_WIDE_RESUME_INSTANCES(MPCG_SEL_RESUME)
MPCG_WIDE_WARM_INSTANCES(MPCG_SEL_WARM)

}  // namespace mpcg
