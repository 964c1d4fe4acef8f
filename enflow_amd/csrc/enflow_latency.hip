// enflow_latency.hip -- the fused flow kernel (flow_kernel.h) built with 8 waves
// (512 threads) per molecule: the latency instance for batches that leave CUs
// idle.  The 256-thread build runs one 4-wave workgroup per molecule, two per
// CU, each wave taking ceil(tiles / 4) of a molecule-layer's 32-pair edge tiles
// in turn; with fewer molecules than CUs (the stated 1024-molecule batch split
// over 8 GPUs: 128 per GPU) a molecule's serial chain of layers is the whole
// kernel time.  Here each molecule owns a CU with two waves per SIMD: half the
// edge tiles per wave, and the pair build / node phase / update with twice the
// threads, so a layer takes about half as long.  The same device code as the
// 256-thread build (WAVES is a compile-time constant of the TU); every
// reduction keeps a fixed order, so results are deterministic (they may differ
// from the 256-thread build in the last bits: rows that straddle two waves'
// tiles are summed in a different grouping).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "enflow_hip.h"
#include "enflow_timing.h"
#include "enflow_latency.h"

#define WAVES 8
// Every kernel of this TU lives in its own namespace: its template instances
// carry other symbol names than the 256-thread TU's.
namespace enflow_lat {
#include "flow_device.h"
#include "flow_kernel.h"

template <int HH, bool REV, bool VAR>
static void launch_v(int prec, int num_mols, hipStream_t st, const FlowArgs& A) {
  const char* name = REV ? "lf_flow_kernel<rev,lat>" : "lf_flow_kernel<fwd,lat>";
  if (prec == ENFLOW_PREC_F16X3)
    ENFLOW_TIMED(name, st, hipLaunchKernelGGL((lf_flow_kernel<HH, 32, REV, PREC_F16X3, 32, VAR>), dim3(num_mols),
                                              dim3(BLOCK), 0, st, A));
  else if (prec == ENFLOW_PREC_BF16)
    ENFLOW_TIMED(name, st, hipLaunchKernelGGL((lf_flow_kernel<HH, 32, REV, PREC_BF16, 32, VAR>), dim3(num_mols),
                                              dim3(BLOCK), 0, st, A));
  else
    ENFLOW_TIMED(name, st, hipLaunchKernelGGL((lf_flow_kernel<HH, 32, REV, PREC_F32, 32, VAR>), dim3(num_mols),
                                              dim3(BLOCK), 0, st, A));
}

template <int HH, bool REV>
static void launch(int prec, int num_mols, hipStream_t st, const FlowArgs& A) {
  if (prec & ENFLOW_EGCL_VARIANTS) launch_v<HH, REV, true>(prec & 0xff, num_mols, st, A);
  else launch_v<HH, REV, false>(prec, num_mols, st, A);
}
}  // namespace enflow_lat

bool enflow_lat_launch(int H, bool rev, int prec, int num_mols, hipStream_t st, const void* flow_args) {
  const auto& A = *static_cast<const enflow_lat::FlowArgs*>(flow_args);
#ifdef ENFLOW_DEV_ONLY
  if (H != 128 || rev || (prec & ENFLOW_EGCL_VARIANTS)) return false;
  enflow_lat::launch<128, false>(prec, num_mols, st, A);
  return true;
#else
  switch (H) {
    case 32: rev ? enflow_lat::launch<32, true>(prec, num_mols, st, A) : enflow_lat::launch<32, false>(prec, num_mols, st, A); return true;
    case 64: rev ? enflow_lat::launch<64, true>(prec, num_mols, st, A) : enflow_lat::launch<64, false>(prec, num_mols, st, A); return true;
    case 128: rev ? enflow_lat::launch<128, true>(prec, num_mols, st, A) : enflow_lat::launch<128, false>(prec, num_mols, st, A); return true;
    default: return false;
  }
#endif
}

#ifdef ENFLOW_STAMPS
// diagnostic build only: the latency TU's own stamp accumulators
extern "C" int enflow_read_stamps_lat(unsigned long long* host_out, int reset) {
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(enflow_lat::enflow_stamp_acc), sizeof(unsigned long long) * NSTAMP) !=
      hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[NSTAMP] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(enflow_lat::enflow_stamp_acc), z, sizeof(z)) != hipSuccess) return -1;
  }
  return NSTAMP;
}
#endif
