// enflow_coop.hip -- the fused flow kernel (flow_kernel.h) with TWO 8-wave
// workgroups per molecule on two CUs, for batches with at most half as many
// molecules as the device has CUs (the stated 1024-molecule batch split over 8
// GPUs: 128 per GPU).  With one workgroup per molecule such a batch leaves half
// the chip idle and a molecule's edge tiles -- ~2/3 of a layer -- run on one CU.
// Here each workgroup of the pair takes half of every layer's tiles; the pair
// swaps its aggregate rows once per layer through global memory (device-scope
// relaxed atomics and a per-layer flag, flow_kernel.h coop_exchange) and both
// run the pair build, node phase and update on identical data.  Co-residency
// of a pair (the exchange waits for the partner) is what the cooperative launch
// guarantees; the wait is bounded (ENFLOW_ERR_INTERNAL instead of a hang).
// Results are deterministic and may differ from the one-workgroup instances in
// the last bits (the aggregate sums group the pairs differently).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <map>
#include <mutex>
#include "enflow_hip.h"
#include "enflow_timing.h"
#include "enflow_latency.h"

#define WAVES 8
#define ENFLOW_COOP 1
namespace enflow_coop {
#include "flow_device.h"
#include "flow_kernel.h"

// exchange rows per workgroup: 32 atoms x (H + 4) floats (H <= 128) + err / big words
constexpr int XSTRIDE = 32 * (128 + 4) + 64;

struct XBuf {
  float* rows = nullptr;
  uint32_t* flags = nullptr;
  int cap = 0;           // molecules
  uint32_t epoch = 0;    // next launch's base
};
std::mutex g_mu;
std::map<std::pair<int, hipStream_t>, XBuf> g_buf;   // per (device, stream): launches on one stream are ordered

template <int HH, bool REV, int PREC>
static bool launch_p(int num_mols, hipStream_t st, FlowArgs& A) {
  void* args[] = {(void*)&A};
  const char* name = REV ? "lf_flow_kernel<rev,coop>" : "lf_flow_kernel<fwd,coop>";
  hipError_t e = hipSuccess;
  ENFLOW_TIMED(name, st, e = hipLaunchCooperativeKernel((const void*)lf_flow_kernel<HH, 32, REV, PREC, 32, false>,
                                                          dim3(2 * num_mols), dim3(BLOCK), args, 0, st));
  if (e != hipSuccess) (void)hipGetLastError();   // refused (e.g. not co-resident): the caller falls back
  return e == hipSuccess;
}

template <int HH, bool REV>
static bool launch(int prec, int num_mols, hipStream_t st, FlowArgs& A) {
  if (prec == ENFLOW_PREC_F16X3) return launch_p<HH, REV, PREC_F16X3>(num_mols, st, A);
  if (prec == ENFLOW_PREC_BF16) return launch_p<HH, REV, PREC_BF16>(num_mols, st, A);
  return launch_p<HH, REV, PREC_F32>(num_mols, st, A);
}
}  // namespace enflow_coop

static int g_coop_max = -1;
static int g_coop_cus[64];

int enflow_coop_set_max(int max_mols) {
  const int prev = g_coop_max;
  g_coop_max = max_mols < 0 ? -1 : max_mols;
  return prev;
}

int enflow_coop_max_now(void) {
  if (g_coop_max >= 0) return g_coop_max;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (g_coop_cus[dev] == 0) {
    int cus = 0, coop = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 0;
    if (hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev) != hipSuccess || !coop) cus = 1;
    g_coop_cus[dev] = cus;
  }
  return g_coop_cus[dev] / 2;
}

bool enflow_coop_launch(int H, bool rev, int prec, int num_mols, hipStream_t st, void* flow_args) {
  using namespace enflow_coop;
  auto& A = *static_cast<FlowArgs*>(flow_args);
  if ((prec & ENFLOW_EGCL_VARIANTS) || A.tape != nullptr || num_mols <= 0 || num_mols > enflow_coop_max_now())
    return false;
  if (H != 32 && H != 64 && H != 128) return false;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return false;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lock(g_mu);
  XBuf& B = g_buf[{dev, st}];
  if (B.cap < num_mols) {
    if (B.rows) {
      // the previous buffers may still be in use by launches queued on `st`
      if (hipStreamSynchronize(st) != hipSuccess) return false;
      (void)hipFree(B.rows);
      (void)hipFree(B.flags);
      B = XBuf{};
    }
    const int cap = num_mols < 128 ? 128 : num_mols;
    if (hipMalloc(&B.rows, sizeof(float) * (size_t)cap * 2 * XSTRIDE) != hipSuccess) return false;
    if (hipMalloc(&B.flags, sizeof(uint32_t) * (size_t)cap * 2) != hipSuccess) {
      (void)hipFree(B.rows);
      B.rows = nullptr;
      return false;
    }
    if (hipMemsetAsync(B.flags, 0, sizeof(uint32_t) * (size_t)cap * 2, st) != hipSuccess) return false;
    B.cap = cap;
    B.epoch = 1;
  }
  A.xchg = B.rows;
  A.xflag = B.flags;
  A.coop_stride = XSTRIDE;
  A.epoch = B.epoch;
  bool ok = false;
#ifdef ENFLOW_DEV_ONLY
  if (H != 128 || rev) return false;
  ok = enflow_coop::launch<128, false>(prec, num_mols, st, A);
#else
  switch (H) {
    case 32: ok = rev ? launch<32, true>(prec, num_mols, st, A) : launch<32, false>(prec, num_mols, st, A); break;
    case 64: ok = rev ? launch<64, true>(prec, num_mols, st, A) : launch<64, false>(prec, num_mols, st, A); break;
    default: ok = rev ? launch<128, true>(prec, num_mols, st, A) : launch<128, false>(prec, num_mols, st, A); break;
  }
#endif
  // flag values of this launch: epoch + 1 .. epoch + n_layers (wrap-safe compares)
  if (ok) B.epoch += (uint32_t)A.n_layers + 2u;
  return ok;
}
