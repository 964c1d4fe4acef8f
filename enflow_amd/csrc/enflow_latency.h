// enflow_latency.h -- entry of the latency build of the fused flow kernel
// (enflow_latency.hip) for the 256-thread TU's dispatch (enflow_flow.hip).
#pragma once
#include <hip/hip_runtime.h>

// Launch lf_flow_kernel with 8 waves per molecule for <= 32-atom molecules.
// `flow_args` points to the caller's FlowArgs (the same struct definition,
// flow_device.h).  Returns false when no latency instance exists for (H, prec).
bool enflow_lat_launch(int H, bool rev, int prec, int num_mols, hipStream_t st, const void* flow_args);

// Launch the cooperative instance (enflow_coop.hip: two 8-wave workgroups per
// <= 32-atom molecule on two CUs, both resident by hipLaunchCooperativeKernel)
// for default-flag layers and inference launches (no training tape).  `A` is
// completed with the stream's exchange buffer and epoch.  Returns false (nothing
// launched) when the instance does not apply or the launch is refused; the
// caller then runs another instance.
bool enflow_coop_launch(int H, bool rev, int prec, int num_mols, hipStream_t st, void* flow_args);
// molecules up to which launch_flow tries the cooperative instance (-1: half
// the device's CUs, the default; 0: never)
int enflow_coop_set_max(int max_mols);
int enflow_coop_max_now(void);
