// enflow_split.h -- entry of the feature-split latency instance of the fused
// flow kernel (enflow_split.hip) for the 256-thread TU's dispatch (enflow_flow.hip).
#pragma once
#include <hip/hip_runtime.h>

// Launch lf_fs_kernel (H = 128, f16x3, inference) when the batch leaves CUs
// idle: two workgroups per molecule (SPLIT = 2) for at most CUs / 2 molecules,
// one (SPLIT = 1) below enflow_set_fs_threshold's bound.  `flow_args` points to
// the caller's FlowArgs (flow_device.h).  Returns false when the instance does
// not apply (the caller launches a whole-tile instance).
bool enflow_fs_launch(int H, bool rev, int prec, int num_mols, hipStream_t st, const void* flow_args);
// the SPLIT this batch would get (0: not this instance)
int enflow_fs_split_for(int num_mols);
