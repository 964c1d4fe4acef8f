// enflow_latency.h -- entry of the latency build of the fused flow kernel
// (enflow_latency.hip) for the 256-thread TU's dispatch (enflow_flow.hip).
#pragma once
#include <hip/hip_runtime.h>

// Launch lf_flow_kernel with 8 waves per molecule for <= 32-atom molecules.
// `flow_args` points to the caller's FlowArgs (the same struct definition,
// flow_device.h).  Returns false when no latency instance exists for (H, prec).
bool enflow_lat_launch(int H, bool rev, int prec, int num_mols, hipStream_t st, const void* flow_args);
