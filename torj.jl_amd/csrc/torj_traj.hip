// torj_traj.hip -- the split pipeline's trajectory kernel k_traj_cell in a
// translation unit of its own, compiled without machine-level loop-invariant
// code motion (csrc/Makefile TRAJ_FLAGS): torj_hip.hip up to its trajectory
// kernels, and their instances.  See the note at the top of torj_hip.hip.
#define TORJ_TRAJ_TU 1
#include "torj_hip.hip"

template __global__ void k_traj_cell<kDepoSamples, true>(TraceArgs, SplitArgs);
template __global__ void k_traj_cell<kDepoSamples, false>(TraceArgs, SplitArgs);
template __global__ void k_traj_cell<kDepoBinned, true>(TraceArgs, SplitArgs);
template __global__ void k_traj_cell<kDepoBinned, false>(TraceArgs, SplitArgs);
template __global__ void k_traj_cell<kDepoNone, true>(TraceArgs, SplitArgs);
template __global__ void k_traj_cell<kDepoNone, false>(TraceArgs, SplitArgs);
