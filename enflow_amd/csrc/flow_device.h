// flow_device.h -- device code shared by the forward (enflow_flow.hip) and
// backward (enflow_backward.hip) translation units: packed-weight layouts,
// MFMA / DPP helpers, the per-molecule LDS image, the neighbour-pair build,
// the EGCL edge tiles and node phase.  Included by exactly those two files.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <type_traits>

#include "enflow_hip.h"
#include "enflow_timing.h"

#define ENFLOW_ABI 13
#ifndef WAVES
#define WAVES 4    // waves per workgroup (the latency build, enflow_latency.hip, uses 8)
#endif
#define BLOCK (64 * WAVES)
// node feature capacity: 8 in libenflow_hip.so; libenflow_hip_nf16.so is the
// same sources built with -DENFLOW_NFMAX=16 (node_nf 9..16).  Only 8 and 16:
// the F16X3 GEMM0 / node-phase k-slices hold 8 features per lane half.
#ifndef ENFLOW_NFMAX
#define ENFLOW_NFMAX 8
#endif
#define NFMAX ENFLOW_NFMAX
static_assert(NFMAX == 8 || NFMAX == 16, "ENFLOW_NFMAX must be 8 or 16");
#define KS0MAX (NFMAX / 8 + 1)   // F16X3 GEMM0 k-slices (feature chunks of 8, + radial)
#ifndef ENFLOW_MSG_MFMA
#define ENFLOW_MSG_MFMA 1  // 1: split-precision message segment sums as selection-matrix MFMAs (edge_tiles)
#endif
#ifndef ENFLOW_MSG_LDS
#define ENFLOW_MSG_LDS 0   // 1: message segment sums through a per-wave LDS scratch instead of DPP
                           // scans (measured 10 % slower: the serial reduce exposes LDS latency)
#endif
#define NFP (NFMAX + 1)  // LDS row stride of h / g / G (odd -> conflict-free across atoms)
#ifndef ENFLOW_WAVES_PER_SIMD
#define ENFLOW_WAVES_PER_SIMD 2   // workgroups of 4 waves per CU (VGPR budget 256 / 168 for 2 / 3)
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// layouts
// ---------------------------------------------------------------------------
// Row of the 32x32 f32 MFMA accumulator held by register r in lane half hh
// (C/D map col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)).
__host__ __device__ constexpr int rho(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

__host__ __device__ inline int node_ksteps(int H, int nf) { return (H + nf + 1) / 2; }

struct EgclLayout {
  int we1f, we2f, wc1f, wn1h, wn1a, wv1f, wn2f, be1, be2, bc1, wc2, bn1, bv1, wv2, bn2, bv2, watt, batt, vfl,
      scl, we1x, wv1x, wn1hx, wn1ax, wn2x, we2x, wc1x, we2b, wc1b, total;
};

// EGCL constructor variants (enflow/nn/egcl.py:11-17), per packed layer (vfl)
enum { EGCL_ATTENTION = 1, EGCL_NORM_DIFF = 2, EGCL_TANH = 4 };

// GEMM precision of the two H x H edge GEMMs (edge_nn.2, coord_nn.0), the
// flow's dominant work (include/enflow_hip.h ENFLOW_PREC_*):
//   PREC_F32   v_mfma_f32_32x32x2_f32 (exact fp32 FMA chain)
//   PREC_F16X3 operands split x = hi + lo in fp16 (weights pre-scaled by a
//              power of two so their lo parts stay normal), three products
//              hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_f16, fp32
//              accumulation: ~22-bit products at 16x the f32 MFMA rate / 3
//   PREC_BF16  bf16 operands, one v_mfma_f32_32x32x16_bf16, fp32 accumulation
enum { PREC_F32 = 0, PREC_F16X3 = 1, PREC_BF16 = 2 };

// Packed EGCL layer (floats).  *f / wn1h / wn1a sections are MFMA A-fragments
// (32x32x2 f32: lane l supplies A[l & 31][k = l >> 5]).  The layout does not
// depend on nf (features beyond nf are zero-padded), only its values do.
__host__ __device__ inline EgclLayout egcl_layout(int H, int nf) {
  (void)nf;
  const int NT = H / 32;
  EgclLayout L;
  int o = 0;
  L.we1f = o; o += NT * (NFMAX + 1) * 64;  // [t][slot][lane]: h_i pairs, h_j pairs, radial
  L.we2f = o; o += H * H;                  // [tp][t][rg][lane][4], rho-permuted k
  L.wc1f = o; o += H * H;                  // [tp][t][rg][lane][4], rho-permuted k
  L.wn1h = o; o += NT * (NFMAX / 2) * 64;  // [tp][s][lane]: node_nn.0, h part
  L.wn1a = o; o += NT * (H / 8) * 256;     // [tp][sg][lane][4]: node_nn.0, agg part
  L.wv1f = o; o += NT * (NFMAX / 2) * 64;  // [tp][s][lane]: vel_scaling_nn.0
  L.wn2f = o; o += NT * 4 * 256;           // [tp][rg][lane][4]: node_nn.2, rho-permuted k
  L.be1 = o; o += H;
  L.be2 = o; o += H;
  L.bc1 = o; o += H;
  L.wc2 = o; o += H;
  L.bn1 = o; o += H;
  L.bv1 = o; o += H;
  L.wv2 = o; o += H;
  L.bn2 = o; o += NFMAX;
  L.bv2 = o; o += 4;
  L.watt = o; o += H;                      // att_nn.0.weight (attention layers; else zeros)
  L.batt = o; o += 4;                      // att_nn.0.bias
  L.vfl = o; o += 4;                       // EGCL_* flags of the layer, act_fn kind, p0, p1 (as floats)
  L.scl = o; o += 16;                      // (2^s, 2^-s) of edge_nn.2, coord_nn.0, edge_nn.0,
                                           // vel_scaling_nn.0, node_nn.0, node_nn.2 (F16X3)
  o = (o + 63) & ~63;
  L.we1x = o; o += NT * KS0MAX * 512;      // [t][ks][lane][hi 8 | lo 8] f16, k = raw column of edge_nn.0
  L.wv1x = o; o += NT * 512;               // [tp][lane][hi|lo]: vel_scaling_nn.0, k = h feature
  L.wn1hx = o; o += NT * 512;              // [tp][lane][hi|lo]: node_nn.0 h part
  L.wn1ax = o; o += NT * (H / 16) * 512;   // [tp][ks][lane][hi|lo]: node_nn.0 agg part, k = 16 ks + 8 kh + j
  L.wn2x = o; o += NT * 2 * 512;           // [tp][s][lane][hi|lo]: node_nn.2, A[q][32 tp + rho(8 s + j, kh)]
  L.we2x = o; o += H * H;                  // [tp][t][s][lane][hi 8 x f16 | lo 8 x f16]
  L.wc1x = o; o += H * H;
  L.we2b = o; o += H * H / 2;              // [tp][t][s][lane][8 x bf16]
  L.wc1b = o; o += H * H / 2;
  o = (o + 63) & ~63;
  L.total = o;
  return L;
}

// F16X3 edge_nn.0 (GEMM0) k order, chosen so each lane half reads ONE atom's
// zero-padded feature row: k-slice ks < nch = ceil(nf / 8) holds features
// 8 ks .. 8 ks + 7 of h_i (lane half 0) and of h_j (lane half 1); the radial
// takes half 1's slot 7 of the last slice when that slot is padding (nf % 8 !=
// 0), else an extra slice of its own (half 0, slot 0).  nf <= 7: one slice
// [h_i[0..7] | h_j[0..6], radial]; nf == 8: [h_i | h_j], [radial, 0..].
// Returns the raw edge_nn.0 input column of (k-slice ks, k = 8 half + slot), or -1.
__host__ __device__ inline int gemm0_nch(int nf) { return (nf + 7) >> 3; }
__host__ __device__ inline bool gemm0_radial_slot7(int nf) { return (nf & 7) != 0; }
__host__ __device__ inline int gemm0_col(int ks, int kk, int nf) {
  const int half = kk >> 3, s = kk & 7;
  const int nch = gemm0_nch(nf);
  if (ks < nch) {
    if (half == 1 && s == 7 && ks == nch - 1 && gemm0_radial_slot7(nf)) return 2 * nf;
    const int f = 8 * ks + s;
    if (f >= nf) return -1;
    return half == 0 ? f : nf + f;
  }
  return (ks == nch && kk == 0 && !gemm0_radial_slot7(nf)) ? 2 * nf : -1;
}
__host__ __device__ inline int gemm0_ksteps(int nf) { return gemm0_nch(nf) + (gemm0_radial_slot7(nf) ? 0 : 1); }

struct RawEgcl {  // offsets into the raw (torch) concatenation
  int We1, be1, We2, be2, Wn1, bn1, Wn2, bn2, Wc1, bc1, wc2, Wv1, bv1, Wv2, bv2, total;
  // training backward (layers_raw / grad_layers): att_nn.0.weight, att_nn.0.bias
  // appended to every layer (unused without attention); stride total_bwd
  int watt, batt, total_bwd;
};
__host__ __device__ inline RawEgcl raw_egcl(int H, int nf) {
  RawEgcl R;
  int o = 0;
  R.We1 = o; o += H * (2 * nf + 1);
  R.be1 = o; o += H;
  R.We2 = o; o += H * H;
  R.be2 = o; o += H;
  R.Wn1 = o; o += H * (H + nf);
  R.bn1 = o; o += H;
  R.Wn2 = o; o += nf * H;
  R.bn2 = o; o += nf;
  R.Wc1 = o; o += H * H;
  R.bc1 = o; o += H;
  R.wc2 = o; o += H;
  R.Wv1 = o; o += H * nf;
  R.bv1 = o; o += H;
  R.Wv2 = o; o += H;
  R.bv2 = o; o += 1;
  R.total = o;
  R.watt = o; o += H;
  R.batt = o; o += 1;
  R.total_bwd = o;
  return R;
}

// Backward-only packed EGCL section (floats): transposed fragments for the
// adjoint GEMMs of the edge chain and k-contiguous node weights for the VALU
// node backward (threads over hidden units k read coalesced rows).
struct EgclBwdLayout { int we2T, wc1T, we1T, wv1T, wn1T, scl, we2Tx, wc1Tx, we1Tx, wn2Tx, wvTx, wnhTx, wn1aTx, total; };
__host__ __device__ inline EgclBwdLayout egcl_bwd_layout(int H) {
  const int NT = H / 32;
  EgclBwdLayout L;
  int o = 0;
  L.we2T = o; o += H * H;             // fragments of edge_nn.2.weight^T   (as we2f)
  L.wc1T = o; o += H * H;             // fragments of coord_nn.0.weight^T  (as wc1f)
  L.we1T = o; o += NT * 4 * 256;      // [tp][rg][lane][4]: A[q][k] = edge_nn.0.weight[k][q], q < 2nf+1
  L.wv1T = o; o += NFMAX * H;         // [f][k] = vel_scaling_nn.0.weight[k][f]
  L.wn1T = o; o += (NFMAX + H) * H;   // [f][k] = node_nn.0.weight[k][f] (rows NFMAX.. = agg part)
  L.scl = o; o += 16;                 // the forward's F16X3 scales (same matrices, same maxima)
  o = (o + 63) & ~63;
  L.we2Tx = o; o += H * H;            // F16X3 fragments of edge_nn.2.weight^T  (as we2x)
  L.wc1Tx = o; o += H * H;            // F16X3 fragments of coord_nn.0.weight^T (as wc1x)
  L.we1Tx = o; o += NT * 2 * 512;     // [tp][s][lane][hi|lo]: A[q][32 tp + rho(8 s + j, kh)] = We1[k][q]
  // node-MLP backward (atoms on the lanes), F16X3 [..][lane][hi 8 | lo 8]:
  L.wn2Tx = o; o += NT * 512;         // [tp]: A[m][q] = node_nn.2.weight[q][32 tp + m], q = 8 kh + j < nf
  L.wvTx = o; o += NT * 2 * 512;      // [tp][s]: A[f][32 tp + rho(8 s + j, kh)] = vel_scaling_nn.0.weight[k][f]
  L.wnhTx = o; o += NT * 2 * 512;     // [tp][s]: the same for node_nn.0.weight[k][f], f < nf
  L.wn1aTx = o; o += NT * (H / 16) * 512;   // [tp][ks]: A[m][k] = node_nn.0.weight[k][nf + 32 tp + m], k = 16 ks + 8 kh + j
  o = (o + 63) & ~63;
  L.total = o;
  return L;
}

// Training tape written by the forward (one block per quantity, layer-major):
// per layer l and atom a the layer INPUT state and what the backward re-reads.
struct TapeLayout { size_t hx, g, pos, vel, q, pairs, cnt, total; int ldhx; };
// the fused forward's pair words of a layer, per molecule a slab of TAPE_PAIR_CAP
// words per atom from its first atom's (a molecule of n <= 64 atoms has at most
// n (n - 1) unique pairs), and the per-row edge counts: the layer backward reads
// them instead of rebuilding the neighbour list from the same positions
constexpr int TAPE_PAIR_CAP = 63;
__host__ __device__ inline TapeLayout tape_layout(int num_atoms, int nf, int H, int n_layers) {
  TapeLayout T;
  const size_t LA = (size_t)num_atoms * n_layers;
  T.ldhx = nf + H;
  size_t o = 0;
  T.hx = o; o += LA * (nf + H);   // [l][a][h (nf) | message sums (H)]  (X of node_nn.0's gradient)
  T.g = o; o += LA * nf;
  T.pos = o; o += LA * 3;
  T.vel = o; o += LA * 3;
  T.q = o; o += LA;               // Q = vel_scaling_nn(h)
  T.pairs = o; o += LA * TAPE_PAIR_CAP;   // [l][a0 .. a0 + n)'s slab: pair words (uint32 bits)
  T.cnt = o; o += LA;             // [l][a]: edges of row a (int32 bits)
  T.total = o;
  return T;
}

// Power-of-two scales for the F16X3 fragments of edge_nn.2, coord_nn.0,
// edge_nn.0, vel_scaling_nn.0, node_nn.0, node_nn.2 (pairs (2^s, 2^-s) at
// scl[0..11]): 2^s with max|W| 2^s in [2^13, 2^14), so hi parts stay far below
// the fp16 maximum and lo parts of typical weights stay normal.  Run by one
// 256-thread block.
// Power-of-two scale of weight matrix k (We2, Wc1, We1, Wv1, Wn1, Wn2) for the
// F16X3 fragments: one workgroup per matrix (launch with a grid of 6).
__device__ __forceinline__ void egcl_scales_block(const float* __restrict__ raw, int H, int nf, float* __restrict__ scl) {
  const RawEgcl R = raw_egcl(H, nf);
  const int k = blockIdx.x;
  const int off[6] = {R.We2, R.Wc1, R.We1, R.Wv1, R.Wn1, R.Wn2};
  const int cnt[6] = {H * H, H * H, H * (2 * nf + 1), H * nf, H * (H + nf), nf * H};
  __shared__ float red[256];
  float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;
  const float* src = raw + off[k];
  const int c = cnt[k];
  int i = threadIdx.x;
  for (; i + 768 < c; i += 1024) {
    m0 = fmaxf(m0, fabsf(src[i]));
    m1 = fmaxf(m1, fabsf(src[i + 256]));
    m2 = fmaxf(m2, fabsf(src[i + 512]));
    m3 = fmaxf(m3, fabsf(src[i + 768]));
  }
  for (; i < c; i += 256) m0 = fmaxf(m0, fabsf(src[i]));
  red[threadIdx.x] = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3));
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float mx = red[0];
    int ex = 0;
    if (mx > 0.f && isfinite(mx)) {
      frexpf(mx, &ex);              // mx = f 2^ex, f in [0.5, 1)
      ex = 14 - ex;                 // mx 2^(14 - ex) in [2^13, 2^14)
      ex = ex > 60 ? 60 : (ex < -60 ? -60 : ex);
    }
    scl[2 * k] = ldexpf(1.f, ex);
    scl[2 * k + 1] = ldexpf(1.f, -ex);
  }
}

// hi / lo fp16 pair of w (already scaled), packed as the two halves of a dword
__device__ __forceinline__ uint32_t f16_split_bits(float w0, float w1, bool lo) {
  const _Float16 h0 = (_Float16)w0, h1 = (_Float16)w1;
  const _Float16 p0 = lo ? (_Float16)(w0 - (float)h0) : h0;
  const _Float16 p1 = lo ? (_Float16)(w1 - (float)h1) : h1;
  return (uint32_t)__builtin_bit_cast(uint16_t, p0) | ((uint32_t)__builtin_bit_cast(uint16_t, p1) << 16);
}

struct AmLayout { int wa1t, ba1, wa2, ba2, act, total; };
__host__ __device__ inline AmLayout argmax_layout(int H, int nf) {
  AmLayout L;
  int o = 0;
  L.wa1t = o; o += nf * H;   // [q][k]
  L.ba1 = o; o += H;
  L.wa2 = o; o += 2 * nf * H; // [o][k] (torch layout)
  L.ba2 = o; o += 2 * NFMAX;
  L.act = o; o += 4;          // activation of network.1: kind, p0, p1 (argmax_raw_act)
  o = (o + 63) & ~63;
  L.total = o;
  return L;
}

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t weights_rsrc(const float* p, int nfloats) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, nfloats * 4, 0x00020000);
}
// voffset: per-lane bytes (VGPR), soffset: uniform bytes (SGPR, usually a constant)
__device__ __forceinline__ float bload(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ f32x4 bload4(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

#ifndef ENFLOW_STORE_AUX
#define ENFLOW_STORE_AUX 0   // cache policy of streamed row stores (gfx950 CPol bits: sc0 1, nt 2, sc1 16)
#endif
__device__ __forceinline__ void bstore(rsrc_t r, int voff, int soff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, soff, ENFLOW_STORE_AUX);
}
__device__ __forceinline__ rsrc_t rows_rsrc(float* p, size_t nfloats) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(nfloats * 4), 0x00020000);
}

__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

__device__ __forceinline__ float sigm_f(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float silu_f(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));   // v_rcp_f32 (1 ulp), not an IEEE divide
}

// silu of 4 independent values in lock-step (mul, exp, add, rcp, mul x 4): every
// transcendental result is consumed 4 instructions later, so no s_nop pads the
// trans-use hazard (the compiler's per-element chains got one after each exp /
// rcp).  Same arithmetic as silu_f.
#ifndef ENFLOW_SILU4_ASM
#define ENFLOW_SILU4_ASM 1
#endif
__device__ __forceinline__ f32x4 silu4(f32x4 z) {
#if ENFLOW_SILU4_ASM
  // first reads of z in compiler code (see silu4s: MFMA-result hazards)
  float t0 = z[0] * -1.4426950408889634f, t1 = z[1] * -1.4426950408889634f, t2 = z[2] * -1.4426950408889634f,
        t3 = z[3] * -1.4426950408889634f;
  f32x4 y;
  asm("v_exp_f32 %4, %4\n\t"
      "v_exp_f32 %5, %5\n\t"
      "v_exp_f32 %6, %6\n\t"
      "v_exp_f32 %7, %7\n\t"
      "v_add_f32 %4, 1.0, %4\n\t"
      "v_add_f32 %5, 1.0, %5\n\t"
      "v_add_f32 %6, 1.0, %6\n\t"
      "v_add_f32 %7, 1.0, %7\n\t"
      "v_rcp_f32 %4, %4\n\t"
      "v_rcp_f32 %5, %5\n\t"
      "v_rcp_f32 %6, %6\n\t"
      "v_rcp_f32 %7, %7\n\t"
      "v_mul_f32 %0, %8, %4\n\t"
      "v_mul_f32 %1, %9, %5\n\t"
      "v_mul_f32 %2, %10, %6\n\t"
      "v_mul_f32 %3, %11, %7\n\t"
      "s_nop 1"
      : "=&v"(y[0]), "=&v"(y[1]), "=&v"(y[2]), "=&v"(y[3]), "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3)
      : "v"(z[0]), "v"(z[1]), "v"(z[2]), "v"(z[3]));
  return y;
#else
  return (f32x4){silu_f(z[0]), silu_f(z[1]), silu_f(z[2]), silu_f(z[3])};
#endif
}
// silu(x * s + b), 4 lanes of a register quad
__device__ __forceinline__ f32x4 silu4_fma(float x0, float x1, float x2, float x3, float s, f32x4 b) {
  return silu4((f32x4){fmaf(x0, s, b[0]), fmaf(x1, s, b[1]), fmaf(x2, s, b[2]), fmaf(x3, s, b[3])});
}

// silu(z) of a scaled pre-activation a = K z (bias already inside a): with
// c = -log2(e) / K,  silu(z) = a / (K + K 2^(a c))  -- mul, exp, fma, rcp, mul:
// the power-of-two weight scale K and the bias cost no instruction of their own
__device__ __forceinline__ float silu_sc(float a, float c, float K) {
  return a * __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_exp2f(a * c), K, K));
}
#ifndef ENFLOW_SILU4S_ASM
#define ENFLOW_SILU4S_ASM 1
#endif
__device__ __forceinline__ f32x4 silu4s(f32x4 a, float c, float K) {
#if ENFLOW_SILU4S_ASM
  // a is usually an MFMA accumulator: its first readers (the scaled arguments)
  // are compiler code, so hipcc pads the MFMA-result -> VALU read hazard; an asm
  // statement gets no such pad (cdna_hip_programming.md §5.7 item 2) and read
  // the accumulators before the chain's last MFMA had landed.  The asm reads a
  // again only in its last multiply, after those reads.
  float t0 = a[0] * c, t1 = a[1] * c, t2 = a[2] * c, t3 = a[3] * c;
  f32x4 y;
  asm("v_exp_f32 %4, %4\n\t"
      "v_exp_f32 %5, %5\n\t"
      "v_exp_f32 %6, %6\n\t"
      "v_exp_f32 %7, %7\n\t"
      "v_fma_f32 %4, %4, %12, %12\n\t"
      "v_fma_f32 %5, %5, %12, %12\n\t"
      "v_fma_f32 %6, %6, %12, %12\n\t"
      "v_fma_f32 %7, %7, %12, %12\n\t"
      "v_rcp_f32 %4, %4\n\t"
      "v_rcp_f32 %5, %5\n\t"
      "v_rcp_f32 %6, %6\n\t"
      "v_rcp_f32 %7, %7\n\t"
      "v_mul_f32 %0, %8, %4\n\t"
      "v_mul_f32 %1, %9, %5\n\t"
      "v_mul_f32 %2, %10, %6\n\t"
      "v_mul_f32 %3, %11, %7\n\t"
      "s_nop 1"   // an fp32 chain's MFMA may read y as its B operand next
      : "=&v"(y[0]), "=&v"(y[1]), "=&v"(y[2]), "=&v"(y[3]), "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "s"(K));
  return y;
#else
  return (f32x4){silu_sc(a[0], c, K), silu_sc(a[1], c, K), silu_sc(a[2], c, K), silu_sc(a[3], c, K)};
#endif
}

// ---------------------------------------------------------------------------
// act_fn of EGCL / ArgMax (enflow/nn/egcl.py:11, enflow/nn/argmax.py:7): the
// reference takes any torch activation module.  Kind + two parameters, packed
// with the layer (EgclLayout::vfl + 1, AmLayout::act).  Only the variant-capable
// (VAR) kernel instances read them; the default instances are SiLU by
// construction, so their code is unchanged.  Definitions and derivatives (at
// the kinks as torch's backward formulas take them):
//   relu        max(z, 0)                        d = z > 0
//   leaky_relu  z > 0 ? z : p0 z                 d = z > 0 ? 1 : p0
//   elu         z > 0 ? z : p0 (e^z - 1)         d = z > 0 ? 1 : p0 e^z
//   celu        z > 0 ? z : p0 (e^(z/p0) - 1)    d = z > 0 ? 1 : e^(z/p0)
//   selu        s (z > 0 ? z : a (e^z - 1))      d = s (z > 0 ? 1 : a e^z)
//   gelu        z Phi(z) (erf)                   d = Phi(z) + z phi(z)
//   gelu_tanh   z (1 + tanh(u)) / 2, u = c (z + 0.044715 z^3)
//   tanh, sigmoid, identity
//   softplus    beta = p0, threshold = p1: z beta > p1 ? z : log1p(e^(beta z)) / beta
//   mish        z tanh(softplus(z))
//   hardtanh    clamp(z, p0, p1)                 d = p0 < z < p1
// ---------------------------------------------------------------------------
enum { ACT_SILU = 0, ACT_RELU = 1, ACT_LEAKY_RELU = 2, ACT_ELU = 3, ACT_CELU = 4, ACT_SELU = 5, ACT_GELU = 6,
       ACT_GELU_TANH = 7, ACT_TANH = 8, ACT_SIGMOID = 9, ACT_SOFTPLUS = 10, ACT_MISH = 11, ACT_HARDTANH = 12,
       ACT_IDENTITY = 13, ACT_COUNT = 14 };
struct Act {
  int k;
  float p0, p1;
};
__host__ __device__ constexpr Act act_silu() { return Act{ACT_SILU, 0.f, 0.f}; }
__device__ __forceinline__ Act act_of(const float* __restrict__ p) {
  return Act{(int)p[0], p[1], p[2]};
}
__device__ __forceinline__ float sigm_exact(float x) { return 1.f / (1.f + expf(-x)); }
// Out of line: inlined at every site of the unrolled tile code the switch
// exceeds hipcc's unroll budget (register arrays then fall back to scratch);
// as calls, the generic path costs a call per element and the SiLU path nothing.
__device__ __attribute__((noinline)) float act_f(const Act& A, float z) {
  switch (A.k) {
    case ACT_RELU: return z < 0.f ? 0.f : z;   // NaN stays NaN (torch.relu)
    case ACT_LEAKY_RELU: return z > 0.f ? z : A.p0 * z;
    case ACT_ELU: return z > 0.f ? z : A.p0 * expm1f(z);
    case ACT_CELU: return z > 0.f ? z : A.p0 * expm1f(z / A.p0);
    case ACT_SELU: return 1.0507009873554805f * (z > 0.f ? z : 1.6732632423543772f * expm1f(z));
    case ACT_GELU: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
    case ACT_GELU_TANH: {
      const float u = 0.79788456080286536f * (z + 0.044715f * z * z * z);
      return 0.5f * z * (1.f + tanhf(u));
    }
    case ACT_TANH: return tanhf(z);
    case ACT_SIGMOID: return sigm_exact(z);
    case ACT_SOFTPLUS: return z * A.p0 > A.p1 ? z : log1pf(expf(A.p0 * z)) / A.p0;
    case ACT_MISH: return z * tanhf(z > 20.f ? z : log1pf(expf(z)));
    case ACT_HARDTANH: return __builtin_isnan(z) ? z : fminf(fmaxf(z, A.p0), A.p1);   // NaN stays NaN
    case ACT_IDENTITY: return z;
    default: return z * sigm_exact(z);   // ACT_SILU
  }
}
__device__ __attribute__((noinline)) float act_d(const Act& A, float z) {
  switch (A.k) {
    case ACT_RELU: return z <= 0.f ? 0.f : 1.f;   // threshold_backward: where(z <= 0, 0, grad)
    case ACT_LEAKY_RELU: return z > 0.f ? 1.f : A.p0;
    case ACT_ELU: return z > 0.f ? 1.f : A.p0 * expf(z);
    case ACT_CELU: return z > 0.f ? 1.f : expf(z / A.p0);
    case ACT_SELU: return 1.0507009873554805f * (z > 0.f ? 1.f : 1.6732632423543772f * expf(z));
    case ACT_GELU:
      return 0.5f * (1.f + erff(z * 0.70710678118654752f)) + z * 0.39894228040143268f * expf(-0.5f * z * z);
    case ACT_GELU_TANH: {
      const float u = 0.79788456080286536f * (z + 0.044715f * z * z * z);
      const float th = tanhf(u);
      return 0.5f * (1.f + th) + 0.5f * z * (1.f - th * th) * 0.79788456080286536f * (1.f + 0.134145f * z * z);
    }
    case ACT_TANH: { const float th = tanhf(z); return 1.f - th * th; }
    case ACT_SIGMOID: { const float s = sigm_exact(z); return s * (1.f - s); }
    case ACT_SOFTPLUS: return z * A.p0 > A.p1 ? 1.f : sigm_exact(A.p0 * z);
    case ACT_MISH: {
      const float sp = z > 20.f ? z : log1pf(expf(z)), th = tanhf(sp);
      return th + z * sigm_exact(z) * (1.f - th * th);
    }
    case ACT_HARDTANH: return (z <= A.p0 || z >= A.p1) ? 0.f : 1.f;   // hardtanh_backward's mask
    case ACT_IDENTITY: return 1.f;
    default: { const float s = sigm_exact(z); return s * (1.f + z * (1.f - s)); }
  }
}
// the kernels' SiLU forms where the instance is SiLU-only (GEN false) or the
// layer's act is SiLU; the generic definition otherwise (wave-uniform branch)
template <bool GEN>
__device__ __forceinline__ float act_v(const Act& A, float z) {
  if (!GEN || A.k == ACT_SILU) return silu_f(z);
  return act_f(A, z);
}
// act(z) and act'(z) together (SiLU: one sigmoid for both, as the backward's
// original forms: f = z s, d = s (1 + z (1 - s)))
template <bool GEN>
__device__ __forceinline__ void act_fd(const Act& A, float z, float& f, float& d) {
  if (!GEN || A.k == ACT_SILU) {
    const float s = __builtin_amdgcn_rcpf(1.0f + __expf(-z));
    f = z * s;
    d = s * (1.f + z * (1.f - s));
  } else {
    f = act_f(A, z);
    d = act_d(A, z);
  }
}
// 4 scaled pre-activations a = K z of an MFMA chain (silu4s's contract); ik = 1 / K
template <bool GEN>
__device__ __forceinline__ f32x4 act4s(f32x4 a, float c, float K, float ik, const Act& A) {
  if (!GEN || A.k == ACT_SILU) return silu4s(a, c, K);
  return (f32x4){act_f(A, a[0] * ik), act_f(A, a[1] * ik), act_f(A, a[2] * ik), act_f(A, a[3] * ik)};
}
template <bool GEN>
__device__ __forceinline__ float act_sc(float a, float c, float K, float ik, const Act& A) {
  if (!GEN || A.k == ACT_SILU) return silu_sc(a, c, K);
  return act_f(A, a * ik);
}

__device__ __forceinline__ float pbc1(float x, float b) { return x - rintf(x / b) * b; }

// torch.clamp(x, -100, 100) (egcl.py:72): NaN passes through, as in torch
// (fminf / fmaxf alone would map a NaN to a bound)
__device__ __forceinline__ float clamp100(float x) {
  return __builtin_isnan(x) ? x : fminf(fmaxf(x, -100.f), 100.f);
}

__device__ __forceinline__ float softplus_f(float x) { return x > 20.f ? x : log1pf(expf(x)); }
__device__ __forceinline__ float logsigmoid_f(float x) { return fminf(x, 0.f) - log1pf(expf(-fabsf(x))); }

// A wave's own LDS traffic is FIFO; this keeps the compiler from moving LDS
// accesses across the point and drains outstanding ones.
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// DPP moves (VALU, no LDS): row_shr:n = 0x110 + n, row_bcast:15 = 0x142, row_bcast:31 = 0x143.
// Lanes whose source is outside the 16-lane row (or rows not in ROWMASK) get `old`.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_i(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWMASK, 0xf, false);
}

// inclusive prefix sum over the wave's 64 lanes, DPP only (no LDS round trips)
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += dpp_i<0x111, 0xf>(0, v);
  v += dpp_i<0x112, 0xf>(0, v);
  v += dpp_i<0x114, 0xf>(0, v);
  v += dpp_i<0x118, 0xf>(0, v);
  v += dpp_i<0x142, 0xa>(0, v);
  v += dpp_i<0x143, 0xc>(0, v);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWMASK, 0xf, false));
}

// max over the wave's 64 lanes: DPP within each row of 16 (quad swaps, half-row
// and row mirrors), then the four row maxima read into SGPRs; wave-uniform
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1, 0xf>(v));    // quad_perm [1, 0, 3, 2]
  v = fmaxf(v, dpp_f<0x4E, 0xf>(v));    // quad_perm [2, 3, 0, 1]
  v = fmaxf(v, dpp_f<0x141, 0xf>(v));   // row_half_mirror
  v = fmaxf(v, dpp_f<0x140, 0xf>(v));   // row_mirror
  const int b = __builtin_bit_cast(int, v);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

// Segmented inclusive scan over the 32 pair-lanes of each wave half, for
// contiguous segments (pairs are sorted by row): lane j ends with the sum of
// its segment's values at lanes <= j.  m1..m16: 1.0 where the lane d to the
// left (d = 1, 2, 4, 8, and lane 15 for the upper 16) is in the same segment.
struct SegMasks { float m1, m2, m4, m8, m16; };

__device__ __forceinline__ SegMasks seg_masks(int row) {
  SegMasks M;
  M.m1 = dpp_i<0x111, 0xf>(-0x7fffffff, row) == row ? 1.f : 0.f;
  M.m2 = dpp_i<0x112, 0xf>(-0x7fffffff, row) == row ? 1.f : 0.f;
  M.m4 = dpp_i<0x114, 0xf>(-0x7fffffff, row) == row ? 1.f : 0.f;
  M.m8 = dpp_i<0x118, 0xf>(-0x7fffffff, row) == row ? 1.f : 0.f;
  M.m16 = dpp_i<0x142, 0xa>(-0x7fffffff, row) == row ? 1.f : 0.f;
  return M;
}

// Four independent segmented scans as fused DPP FMAs (v += dpp(v) * mask): 20
// VALU instead of 40 (no separate v_mov_b32_dpp).  The four chains interleave, so
// every DPP source was written >= 3 instructions earlier; the leading s_nop
// covers the write of the inputs by the code before the statement.
__device__ __forceinline__ void seg_scan4(float& a, float& b, float& c, float& d, const SegMasks& M) {
  asm("s_nop 1\n\t"
      "v_fmac_f32_dpp %0, %0, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %1, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %2, %2, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %3, %3, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %0, %5 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %1, %5 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %2, %2, %5 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %3, %3, %5 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %0, %6 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %1, %6 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %2, %2, %6 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %3, %3, %6 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %0, %7 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %1, %7 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %2, %2, %7 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %3, %3, %7 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %0, %8 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %1, %8 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %2, %2, %8 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %3, %3, %8 row_bcast:15 row_mask:0xa bank_mask:0xf"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
      : "v"(M.m1), "v"(M.m2), "v"(M.m4), "v"(M.m8), "v"(M.m16));
}

// The same segmented scan, NaN-exact: each step's shifted copy is moved with
// full EXEC (v_mov_b32_dpp), then added under an EXEC mask of the lanes whose
// source lane is in their segment, so a NaN never leaks into a neighbouring
// segment (the 0 * NaN of the multiplier form would).  2 VALU per value and
// step instead of 1: used where it is cheap (the per-pair forces).
struct SegExec { uint64_t e1, e2, e4, e8, e16; };

__device__ __forceinline__ SegExec seg_exec(int row) {
  SegExec E;
  E.e1 = __ballot(dpp_i<0x111, 0xf>(-0x7fffffff, row) == row);
  E.e2 = __ballot(dpp_i<0x112, 0xf>(-0x7fffffff, row) == row);
  E.e4 = __ballot(dpp_i<0x114, 0xf>(-0x7fffffff, row) == row);
  E.e8 = __ballot(dpp_i<0x118, 0xf>(-0x7fffffff, row) == row);
  E.e16 = __ballot(dpp_i<0x142, 0xa>(-0x7fffffff, row) == row);
  return E;
}

#define ENFLOW_SCANX_STEP(CTRL, MASK)                              \
  "v_mov_b32_dpp %5, %0 " CTRL " bank_mask:0xf\n\t"              \
  "v_mov_b32_dpp %6, %1 " CTRL " bank_mask:0xf\n\t"              \
  "v_mov_b32_dpp %7, %2 " CTRL " bank_mask:0xf\n\t"              \
  "v_mov_b32_dpp %8, %3 " CTRL " bank_mask:0xf\n\t"              \
  "s_mov_b64 exec, " MASK "\n\t"                                 \
  "v_add_f32 %0, %0, %5\n\t"                                     \
  "v_add_f32 %1, %1, %6\n\t"                                     \
  "v_add_f32 %2, %2, %7\n\t"                                     \
  "v_add_f32 %3, %3, %8\n\t"                                     \
  "s_mov_b64 exec, %4\n\t"

__device__ __forceinline__ void seg_scan4x(float& a, float& b, float& c, float& d, const SegExec& E) {
  uint64_t sv;
  float t0, t1, t2, t3;
  asm volatile("s_mov_b64 %4, exec\n\t"
      "s_nop 1\n\t"
      ENFLOW_SCANX_STEP("row_shr:1 row_mask:0xf", "%9")
      ENFLOW_SCANX_STEP("row_shr:2 row_mask:0xf", "%10")
      ENFLOW_SCANX_STEP("row_shr:4 row_mask:0xf", "%11")
      ENFLOW_SCANX_STEP("row_shr:8 row_mask:0xf", "%12")
      ENFLOW_SCANX_STEP("row_bcast:15 row_mask:0xa", "%13")
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=&s"(sv), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3)
      : "s"(E.e1), "s"(E.e2), "s"(E.e4), "s"(E.e8), "s"(E.e16));
}
#undef ENFLOW_SCANX_STEP

__device__ __forceinline__ float seg_scan(float v, const SegMasks& M) {
  v = fmaf(M.m1, dpp_f<0x111, 0xf>(v), v);
  v = fmaf(M.m2, dpp_f<0x112, 0xf>(v), v);
  v = fmaf(M.m4, dpp_f<0x114, 0xf>(v), v);
  v = fmaf(M.m8, dpp_f<0x118, 0xf>(v), v);
  v = fmaf(M.m16, dpp_f<0x142, 0xa>(v), v);
  return v;
}


// Chained GEMM  acc[tp] += W_packed[tp][t][r] * X[t][r]  over all (t, r):
// X is an accumulator-layout register tile (lane = pair, registers = features
// in rho order), W the fragment-packed [H][H] weight.  sched_barrier pins the
// prefetch distance (hipcc otherwise hoists every fragment load: VGPRs).
//  ENFLOW_CHAIN_WIDE=1: steps of NT*4 independent MFMAs (all output tiles),
//                       fragments one step (>= 1024 cycles) ahead;
//  ENFLOW_CHAIN_WIDE=0: one output tile at a time (a dependent MFMA chain runs
//                       at the issue rate for 32x32x2), 3-deep fragment ring.
#ifndef ENFLOW_SEGSCAN_ASM
#define ENFLOW_SEGSCAN_ASM 1
#endif
#ifndef ENFLOW_CHAIN_WIDE
#define ENFLOW_CHAIN_WIDE 1
#endif
template <int NT>
__device__ __forceinline__ void chain_gemm_wide(rsrc_t W, int off_floats, const f32x16 (&X)[NT], f32x16 (&acc)[NT],
                                                int lane) {
  f32x4 cur[NT], nxt[NT];
  const int vo = lane * 16;
#pragma unroll
  for (int tp = 0; tp < NT; ++tp) cur[tp] = bload4(W, vo, (off_floats + (tp * NT) * 4 * 256) * 4);
#pragma unroll
  for (int step = 0; step < NT * 4; ++step) {
    const int t = step >> 2, rg = step & 3;
    if (step + 1 < NT * 4) {
      const int t2 = (step + 1) >> 2, rg2 = (step + 1) & 3;
#pragma unroll
      for (int tp = 0; tp < NT; ++tp) nxt[tp] = bload4(W, vo, (off_floats + ((tp * NT + t2) * 4 + rg2) * 256) * 4);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int tp = 0; tp < NT; ++tp) acc[tp] = mfma32(cur[tp][u], X[t][4 * rg + u], acc[tp]);
    __builtin_amdgcn_sched_barrier(0);
    if (step + 1 < NT * 4) {
#pragma unroll
      for (int tp = 0; tp < NT; ++tp) cur[tp] = nxt[tp];
    }
  }
}

// Same wide chain with a VALU/LDS "filler" interleaved into every step: fill(step)
// must not touch acc; sched_group_barrier asks hipcc to alternate one MFMA with
// up to FPM filler instructions, so the filler issues while the MFMAs execute.
struct NoMid {
  __device__ __forceinline__ void operator()() const {}
};
struct NoLate {
  __device__ __forceinline__ void operator()(int) const {}
};

// mid(): called once (NT == 4 only), outside the MFMA/filler scheduling groups,
// after fillers 0 .. 2 NT - 1 and before filler 2 NT
template <int NT, int FPM, class Fill, class Mid = NoMid>
__device__ __forceinline__ void chain_gemm_fill(rsrc_t W, int off_floats, const f32x16 (&X)[NT], f32x16 (&acc)[NT],
                                                int lane, Fill&& fill, Mid&& mid = NoMid{}) {
  f32x4 cur[NT], nxt[NT];
  const int vo = lane * 16;
#pragma unroll
  for (int tp = 0; tp < NT; ++tp) cur[tp] = bload4(W, vo, (off_floats + (tp * NT) * 4 * 256) * 4);
#pragma unroll
  for (int step = 0; step < NT * 4; ++step) {
    const int t = step >> 2, rg = step & 3;
    if (NT == 4 && step == 8) {
      __builtin_amdgcn_sched_barrier(0);
      mid();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (step + 1 < NT * 4) {
      const int t2 = (step + 1) >> 2, rg2 = (step + 1) & 3;
#pragma unroll
      for (int tp = 0; tp < NT; ++tp) nxt[tp] = bload4(W, vo, (off_floats + ((tp * NT + t2) * 4 + rg2) * 256) * 4);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int tp = 0; tp < NT; ++tp) acc[tp] = mfma32(cur[tp][u], X[t][4 * rg + u], acc[tp]);
    fill(step);
#pragma unroll
    for (int k = 0; k < 4 * NT; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);           // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x002 | 0x100 | 0x200, FPM, 0);   // VALU / DS
    }
    __builtin_amdgcn_sched_barrier(0);
    if (step + 1 < NT * 4) {
#pragma unroll
      for (int tp = 0; tp < NT; ++tp) cur[tp] = nxt[tp];
    }
  }
}

// one output tile: acc += sum_{t, r} W[tp][t][r] X[t][r], fragments 3 steps ahead
template <int NT>
__device__ __forceinline__ f32x16 chain_tile(rsrc_t W, int off_floats, const f32x16 (&X)[NT], f32x16 acc, int tp,
                                             int lane) {
  constexpr int S = NT * 4;
  const int vo = lane * 16;
  f32x4 ring[3];
#pragma unroll
  for (int k = 0; k < 3 && k < S; ++k) ring[k] = bload4(W, vo, (off_floats + (tp * NT * 4 + k) * 256) * 4);
#pragma unroll
  for (int step = 0; step < S; ++step) {
    const int t = step >> 2, rg = step & 3;
    const f32x4 cur = ring[step % 3];
    if (step + 3 < S) ring[step % 3] = bload4(W, vo, (off_floats + (tp * NT * 4 + step + 3) * 256) * 4);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = mfma32(cur[u], X[t][4 * rg + u], acc);
    __builtin_amdgcn_sched_barrier(0);
  }
  return acc;
}

template <int NT>
__device__ __forceinline__ void chain_gemm(rsrc_t W, int off_floats, const f32x16 (&X)[NT], f32x16 (&acc)[NT],
                                           int lane) {
#if ENFLOW_CHAIN_WIDE
  chain_gemm_wide<NT>(W, off_floats, X, acc, lane);
#else
#pragma unroll
  for (int tp = 0; tp < NT; ++tp) acc[tp] = chain_tile<NT>(W, off_floats, X, acc[tp], tp, lane);
#endif
}

// ---- split-precision chains (see PREC_*): same "weights = A, activations = B"
// orientation, k-step s of feature tile t = registers 8s..8s+7 of X[t] (k order
// rho-permuted, folded into the packed fragments).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16 mfma_f16(f32x4 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma_bf16(f32x4 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), b, c, 0, 0, 0);
}
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
// ds_read_b64_tr_b16: per 16-lane group, lane 4q + p addresses row q / columns
// 4p .. 4p + 3 of a 4 x 16 block of 16-bit elements; lane i receives column i
// (element q = row q).  EXEC must be full.
__device__ __forceinline__ s16x4 lds_tr16(const uint32_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
__device__ __forceinline__ f16x8 cat_f16x8(s16x4 a, s16x4 b) {
  return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

// F16X3 small-operand guard.  A split x = hi + lo holds x to fp32 accuracy
// only while lo = x - hi is a normal fp16, i.e. |x| >~ 2^-3: activation
// operands carry no power-of-two scale, so an operand whose values are ALL
// small loses relative accuracy (1e-3: ~1.7e-5 normwise per GEMM).  Per
// molecule (row block) and layer, each GEMM operand kind records whether any
// of its values reached 2^-7 (fp16 exponent field >= 8: bit 13 or 14 of a hi
// half set; OR of the packed hi words, two words per v_or3); a kind that never
// did flags ENFLOW_ERR_RANGE and the host re-runs the launch with fp32 GEMMs.
// Unflagged, the worst case is an operand whose max is just above 2^-7:
// ~2e-6 normwise per GEMM.
#define ENFLOW_BIG_BITS 0x60006000u
enum {
  BIGK_X0 = 1,      // edge_nn.0 input [h_i, h_j, radial]
  BIGK_Y0 = 2,      // edge_nn.2 input act(edge_nn.0 ..)
  BIGK_M = 4,       // coord_nn.0 input (the messages)
  BIGK_HV = 8,      // vel_scaling_nn.0 input h
  BIGK_HA = 16,     // node_nn.0 input [h, agg]
  BIGK_NH = 32,     // node_nn.2 input act(node_nn.0 ..)
  BIGK_EDGE = 64,   // the block ran edge tiles
  BIGK_NODE = 128   // the block ran node items
};
__device__ __forceinline__ uint32_t or_hi(uint32_t acc, const f16x8& bh) {
  const u32x4v v = __builtin_bit_cast(u32x4v, bh);
  return acc | v[0] | v[1] | v[2] | v[3];
}
// the kinds that ran but never saw a value >= 2^-7
__device__ __forceinline__ bool small_operands(uint32_t big) {
  const uint32_t need = ((big & BIGK_EDGE) ? (BIGK_X0 | BIGK_Y0 | BIGK_M) : 0u) |
                        ((big & BIGK_NODE) ? (BIGK_HV | BIGK_HA | BIGK_NH) : 0u);
  return (big & need) != need;
}
// x = hi + lo in fp16.  ENFLOW_SPLIT_MIX: lo = f16(x - hi) by v_fma_mix{lo,hi}_f16
// reading hi straight from its packed fp16 register (x * 1 - hi in one fused
// op, one rounding), 1.5 VALU per element instead of 3 (convert hi back to
// fp32, subtract, convert).
#ifndef ENFLOW_SPLIT_MIX
#define ENFLOW_SPLIT_MIX 1
#endif
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
// The four lo words of a k-slice in ONE statement that ends with `s_nop 1`:
// its last v_fma_mix writes a VGPR an MFMA reads as its B operand, and hipcc
// pads no VALU-write -> MFMA-read hazard (2 wait states) for an asm output
// (cdna_hip_programming.md §5.7 item 2; tools/asm_hazard_scan.py check (b):
// as four statements the large-system kernel read the last word 1 state after
// its write).
#define ENFLOW_MIX2(D, A, B, H)                                                   \
  "v_fma_mixlo_f16 " D ", " A ", 1.0, -" H " op_sel_hi:[0,0,1]\n\t"              \
  "v_fma_mixhi_f16 " D ", " B ", 1.0, -" H " op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
__device__ __forceinline__ void split_lo8(const float (&x)[8], const uint32_t (&h)[4], uint32_t (&l)[4]) {
  asm(ENFLOW_MIX2("%0", "%4", "%5", "%12") ENFLOW_MIX2("%1", "%6", "%7", "%13")
      ENFLOW_MIX2("%2", "%8", "%9", "%14") ENFLOW_MIX2("%3", "%10", "%11", "%15")
      "s_nop 1"
      : "=&v"(l[0]), "=&v"(l[1]), "=&v"(l[2]), "=&v"(l[3])
      : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]),
        "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]));
}
#undef ENFLOW_MIX2
__device__ __forceinline__ void split_f16(const f32x16& X, int s, f16x8& hi, f16x8& lo) {
#if ENFLOW_SPLIT_MIX
  uint32_t h[4], l[4];
  float x[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x[2 * j] = X[8 * s + 2 * j];
    x[2 * j + 1] = X[8 * s + 2 * j + 1];
    const f16x2 hp = {(_Float16)x[2 * j], (_Float16)x[2 * j + 1]};   // v_cvt_pk_f16_f32 (RNE)
    h[j] = __builtin_bit_cast(uint32_t, hp);
  }
  split_lo8(x, h, l);
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  hi = __builtin_bit_cast(f16x8, (u32x4){h[0], h[1], h[2], h[3]});
  lo = __builtin_bit_cast(f16x8, (u32x4){l[0], l[1], l[2], l[3]});
#else
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = X[8 * s + j];
    const _Float16 h = (_Float16)x;
    hi[j] = h;
    lo[j] = (_Float16)(x - (float)h);
  }
#endif
}
__device__ __forceinline__ bf16x8 to_bf16(const f32x16& X, int s) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (__bf16)X[8 * s + j];
  return b;
}

// acc[tp] += W[tp][t] X[t] in F16X3.  A step is one k-slice (t, s) x one group
// of TPG output tiles (3 TPG MFMAs), so only TPG tiles' hi/lo fragments (and
// their prefetch) are live; the operand split of the next k-slice and the
// filler calls (4 NT per GEMM, the fp32 chain's granularity) are interleaved
// between the MFMAs.
#ifndef ENFLOW_FPM1
#define ENFLOW_FPM1 2        // filler instructions per MFMA in GEMM1 (edge_nn.2) / GEMM2 (coord_nn.0)
#endif
#ifndef ENFLOW_FPM2
#define ENFLOW_FPM2 6
#endif
#ifndef ENFLOW_X3_TPG
#define ENFLOW_X3_TPG 1      // output tiles per step (2: 73 VGPR spills in the tile loop since the bias-in-accumulator SiLU)
#endif
#ifndef ENFLOW_X3_DEPTH
#define ENFLOW_X3_DEPTH 2    // fragment ring depth (prefetch distance + 1 steps)
#endif
#ifndef ENFLOW_FWD_X3_DEPTH
#define ENFLOW_FWD_X3_DEPTH 3   // the 4-wave <= 32-atom forward / reverse edge tiles: one L2 round trip more
#endif                          // in flight (+1-2 %, bitwise equal; other instances spill more at 3)
struct NoSplit {
  __device__ __forceinline__ void operator()(int, const f16x8&, const f16x8&) const {}
};
// late(step): called at every step 0 .. S-1 after the fillers (and as late(S),
// late(S + 1) after the chain); onsplit(ts, hi, lo): the split operand of
// k-slice ts (features 16 ts .. 16 ts + 15, rho order), as soon as it exists
// The fragment ring of chain_x3_fill; x3_prologue requests its first D - 1
// steps, which a caller can do well before the chain (chain_x3_fill_r), so that
// L2 round trip overlaps other work instead of opening the chain
template <int NT, int DEP>
struct X3Ring {
  static constexpr int TPG = NT >= ENFLOW_X3_TPG ? ENFLOW_X3_TPG : NT;
  static constexpr int NGR = NT / TPG;
  static constexpr int S = NT * 2 * NGR;
  f32x4 rh[DEP][TPG], rl[DEP][TPG];
  __device__ __forceinline__ static int foff(int off_floats, int step, int q) {
    const int gi = step % NGR, ts = step / NGR;
    const int tp = gi * TPG + q;
    return (off_floats + ((tp * NT + (ts >> 1)) * 2 + (ts & 1)) * 512) * 4;
  }
};
template <int NT, int DEP>
__device__ __forceinline__ void x3_prologue(X3Ring<NT, DEP>& R, rsrc_t W, int off_floats, int lane) {
  using RG = X3Ring<NT, DEP>;
  const int vo = lane * 32;
#pragma unroll
  for (int d = 0; d < DEP - 1; ++d)
    if (d < RG::S) {
#pragma unroll
      for (int q = 0; q < RG::TPG; ++q) {
        R.rh[d][q] = bload4(W, vo, RG::foff(off_floats, d, q));
        R.rl[d][q] = bload4(W, vo + 16, RG::foff(off_floats, d, q));
      }
    }
}
template <int NT, int FPM, int DEP, class Fill, class Mid = NoMid, class Late = NoLate, class Split = NoSplit>
__device__ __forceinline__ void chain_x3_fill_r(rsrc_t W, int off_floats, const f32x16 (&X)[NT], f32x16 (&acc)[NT],
                                                int lane, X3Ring<NT, DEP>& R, Fill&& fill, Mid&& mid = NoMid{},
                                                Late&& late = NoLate{}, Split&& onsplit = NoSplit{});
template <int NT, int FPM, int DEP = ENFLOW_X3_DEPTH, class Fill, class Mid = NoMid, class Late = NoLate,
          class Split = NoSplit>
__device__ __forceinline__ void chain_x3_fill(rsrc_t W, int off_floats, const f32x16 (&X)[NT], f32x16 (&acc)[NT],
                                              int lane, Fill&& fill, Mid&& mid = NoMid{}, Late&& late = NoLate{},
                                              Split&& onsplit = NoSplit{}) {
  X3Ring<NT, DEP> R;
  x3_prologue(R, W, off_floats, lane);
  chain_x3_fill_r<NT, FPM, DEP>(W, off_floats, X, acc, lane, R, fill, mid, late, onsplit);
}
template <int NT, int FPM, int DEP, class Fill, class Mid, class Late, class Split>
__device__ __forceinline__ void chain_x3_fill_r(rsrc_t W, int off_floats, const f32x16 (&X)[NT], f32x16 (&acc)[NT],
                                                int lane, X3Ring<NT, DEP>& R, Fill&& fill, Mid&& mid, Late&& late,
                                                Split&& onsplit) {
  using RG = X3Ring<NT, DEP>;
  constexpr int TPG = RG::TPG;
  constexpr int NGR = RG::NGR;
  constexpr int S = RG::S;
  constexpr int FPS = (4 * NT) / S > 0 ? (4 * NT) / S : 1;
  constexpr int FTOT = 4 * NT;
  constexpr int D = DEP;
  auto& rh = R.rh;
  auto& rl = R.rl;
  const int vo = lane * 32;
  auto foff = [&](int step, int q) { return RG::foff(off_floats, step, q); };
  f16x8 bh, bl;
  split_f16(X[0], 0, bh, bl);
  onsplit(0, bh, bl);
#pragma unroll
  for (int step = 0; step < S; ++step) {
    const int gi = step % NGR;
    const int cur = step % D;
    if (NT == 4 && step * FPS == 2 * NT) {   // fillers 0 .. 2 NT - 1 have run
      __builtin_amdgcn_sched_barrier(0);
      mid();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (step + D - 1 < S) {
      const int sl = (step + D - 1) % D;
#pragma unroll
      for (int q = 0; q < TPG; ++q) {
        rh[sl][q] = bload4(W, vo, foff(step + D - 1, q));
        rl[sl][q] = bload4(W, vo + 16, foff(step + D - 1, q));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < TPG; ++q) acc[gi * TPG + q] = mfma_f16(rh[cur][q], bh, acc[gi * TPG + q]);
#pragma unroll
    for (int q = 0; q < TPG; ++q) acc[gi * TPG + q] = mfma_f16(rh[cur][q], bl, acc[gi * TPG + q]);
#pragma unroll
    for (int q = 0; q < TPG; ++q) acc[gi * TPG + q] = mfma_f16(rl[cur][q], bh, acc[gi * TPG + q]);
#pragma unroll
    for (int f = 0; f < FPS; ++f)
      if (step * FPS + f < FTOT) fill(step * FPS + f);
    late(step);
    f16x8 nbh = bh, nbl = bl;
    if (step + 1 < S && (step + 1) % NGR == 0) {
      const int ts = (step + 1) / NGR;
      split_f16(X[ts >> 1], ts & 1, nbh, nbl);
      onsplit(ts, nbh, nbl);
    }
#pragma unroll
    for (int k = 0; k < 3 * TPG; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002 | 0x100 | 0x200, FPM, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    bh = nbh;
    bl = nbl;
  }
  late(S);
  late(S + 1);
  late(S + 2);
}

// acc[tp] += W[tp][t] X[t] in BF16: 2NT k-steps of NT MFMAs.
// late / onsplit as chain_x3_fill (onsplit(ts): k-slice ts's operand is built)
struct NoSplit1 {
  __device__ __forceinline__ void operator()(int) const {}
};
template <int NT, int FPM, class Fill, class Mid = NoMid, class Late = NoLate, class Split = NoSplit1>
__device__ __forceinline__ void chain_b16_fill(rsrc_t W, int off_floats, const f32x16 (&X)[NT], f32x16 (&acc)[NT],
                                               int lane, Fill&& fill, Mid&& mid = NoMid{}, Late&& late = NoLate{},
                                               Split&& onsplit = NoSplit1{}) {
  constexpr int S = 2 * NT;
  f32x4 cb[NT], nb[NT];
  const int vo = lane * 16;
#pragma unroll
  for (int tp = 0; tp < NT; ++tp) cb[tp] = bload4(W, vo, (off_floats + (tp * NT * 2) * 256) * 4);
  bf16x8 b = to_bf16(X[0], 0);
  onsplit(0);
#pragma unroll
  for (int step = 0; step < S; ++step) {
    if (NT == 4 && step == 4) {
      __builtin_amdgcn_sched_barrier(0);
      mid();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (step + 1 < S) {
      const int t2 = (step + 1) >> 1, s2 = (step + 1) & 1;
#pragma unroll
      for (int tp = 0; tp < NT; ++tp) nb[tp] = bload4(W, vo, (off_floats + ((tp * NT + t2) * 2 + s2) * 256) * 4);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int tp = 0; tp < NT; ++tp) acc[tp] = mfma_bf16(cb[tp], b, acc[tp]);
    fill(2 * step);
    fill(2 * step + 1);
    late(step);
    bf16x8 n2 = b;
    if (step + 1 < S) {
      n2 = to_bf16(X[(step + 1) >> 1], (step + 1) & 1);
      onsplit(step + 1);
    }
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002 | 0x100 | 0x200, 4 * FPM, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    b = n2;
    if (step + 1 < S) {
#pragma unroll
      for (int tp = 0; tp < NT; ++tp) cb[tp] = nb[tp];
    }
  }
  late(S);
  late(S + 1);
  late(S + 2);
}

// GEMM with the precision's chain; off_* are the packed sections of the matrix
template <int PREC, int NT, int FPM, int DEP = ENFLOW_X3_DEPTH, class Fill, class Mid = NoMid, class Split = NoSplit>
__device__ __forceinline__ void chain_prec_fill(rsrc_t W, int off_f32, int off_x3, int off_b16, const f32x16 (&X)[NT],
                                                f32x16 (&acc)[NT], int lane, Fill&& fill, Mid&& mid = NoMid{},
                                                Split&& onsplit = NoSplit{}) {
  if constexpr (PREC == PREC_F16X3) chain_x3_fill<NT, FPM, DEP>(W, off_x3, X, acc, lane, fill, mid, NoLate{}, onsplit);
  else if constexpr (PREC == PREC_BF16) chain_b16_fill<NT, FPM>(W, off_b16, X, acc, lane, fill, mid);
  else chain_gemm_fill<NT, FPM>(W, off_f32, X, acc, lane, fill, mid);
}

// accumulators initialised from a bias image in LDS (acc[t][4 g4 + u] holds
// feature 32 t + 8 g4 + 4 hh + u): the bias enters the MFMA chain, nothing is
// added after it.  The image holds the bias times the weights' power-of-two
// scale, so the chain's result is scale * (W x + b).
template <int NT>
__device__ __forceinline__ void acc_from_bias(f32x16 (&acc)[NT], const float* __restrict__ b, int hh) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 v = ld4(b + 32 * t + 8 * g4 + 4 * hh);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[t][4 * g4 + u] = v[u];
    }
}

// X[t][r] = silu(X[t][r] + bias[32 t + rho(r, hh)]); bias read from LDS as float4
template <int NT>
__device__ __forceinline__ void bias_silu(f32x16 (&X)[NT], const float* __restrict__ bias, int hh) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(bias + 32 * t + 8 * g4 + 4 * hh);
#pragma unroll
      for (int u = 0; u < 4; ++u) X[t][4 * g4 + u] = silu_f(X[t][4 * g4 + u] + b[u]);
      __builtin_amdgcn_sched_barrier(0);
    }
}

// ---------------------------------------------------------------------------
// diagnostic phase stamps (compiled only with -DENFLOW_STAMPS; never in the
// product library): per phase, the summed shader-clock cycles of wave 0 of
// every workgroup, measured between the phase's enclosing barriers.
#if defined(ENFLOW_STAMPS) || (defined(ENFLOW_STAMPS_BWD) && defined(ENFLOW_BACKWARD_TU))
#define NSTAMP 20
__device__ unsigned long long enflow_stamp_acc[NSTAMP];
#define STAMP_DECL unsigned long long st_prev = __builtin_amdgcn_s_memtime(), st_acc[NSTAMP] = {0};
#define STAMP_ARGS , unsigned long long& st_prev, unsigned long long (&st_acc)[NSTAMP]
#define STAMP_PASS , st_prev, st_acc
#define STAMP(k)                                               \
  do {                                                         \
    unsigned long long now_ = __builtin_amdgcn_s_memtime();    \
    st_acc[k] += now_ - st_prev;                               \
    st_prev = now_;                                            \
  } while (0)
#define STAMP_FLUSH                                                              \
  if (threadIdx.x == 0)                                                          \
    for (int k_ = 0; k_ < NSTAMP; ++k_) atomicAdd(&enflow_stamp_acc[k_], st_acc[k_]);
#else
#define STAMP_DECL
#define STAMP_ARGS
#define STAMP_PASS
#define STAMP(k) do {} while (0)
#define STAMP_FLUSH
#endif

// ---------------------------------------------------------------------------
// shared memory
// ---------------------------------------------------------------------------
// RB = rows per block.  RB == NMAX: the whole molecule's pair list and
// aggregates are resident (one block per layer).  RB < NMAX (large molecules):
// per layer the image masks / id_mapping are built for all atoms once, then
// the pair list, edge tiles and node phase run one block of RB rows at a time;
// the finished blocks' forces are parked in F and the leapfrog update runs
// after the last block.
//
// The blocked image is kept under ~72 KB so two workgroups share a CU: 16-bit
// multiplicity counts, a pair buffer of PC entries filled in as many
// compaction passes as a block needs, ArgMax outputs per chunk of RB atoms,
// per-atom boxes read from global memory.
//
// BWD = the training backward's image (enflow_backward.hip): no segment-sum
// buffers, node-phase partials or ArgMax outputs; 16-bit counts; the union
// instead holds a chunk of node-MLP adjoint rows (NBW floats).
template <int H, int NMAX, int RB = NMAX, bool BWD = false>
struct Smem {
  static constexpr int NT = H / 32;
  // agg row: H message sums, 3 force sums.  Forward images: H + 4 floats, rows
  // 16-B aligned so a segment end adds 4 features with one ds_read_b128 /
  // ds_write_b128 at a constant offset (ds_read_b128 banks 4 a + c mod 64: conflict-
  // free over 16 rows); the backward's atom-lane b32 stores keep the odd stride.
  static constexpr int AST = BWD ? H + 3 : H + 4;
  static constexpr bool BLOCKED = RB < NMAX;
  static constexpr bool PACKC = BLOCKED || BWD;                          // 2 x 16-bit counts per word
  static constexpr int MAXP = RB * (NMAX - 1);
  static constexpr int PC = BLOCKED ? 512 : MAXP;                       // pair buffer entries
  static constexpr int CW = PACKC ? (RB * NMAX + 1) / 2 : RB * NMAX;    // count words
  static constexpr int NETA = BWD ? 1 : (BLOCKED ? RB : NMAX);          // ArgMax output rows
  static constexpr int NBCH = 8;                                        // BWD: atoms per node chunk
  // BWD union member: node-chunk adjoint rows, then per-wave edge-adjoint sums
  // ([wave][atom][nf + 3], summed over the waves in a fixed order)
  static constexpr int NBW = BWD ? (NBCH * 2 * H > WAVES * NMAX * (NFMAX + 3) ? NBCH * 2 * H
                                                                             : WAVES * NMAX * (NFMAX + 3))
                                 : 1;
  float pos[NMAX * 3], vel[NMAX * 3], boxa[BLOCKED ? 3 : NMAX * 3];
  float h[NMAX * NFP], g[NMAX * NFP], G[BWD ? 1 : NMAX * NFP];
  float Q[NMAX];
  float F[BLOCKED ? NMAX * 3 : 1];    // forces of finished row blocks (blocked only)
  alignas(16) float bias[4 * H];      // be1, be2, bc1, wc2 of the current layer
  // F16X3 edge_nn.0 fragments of the current layer ([t][ks][hi lanes | lo lanes]
  // x 4 floats) for the <= 32-atom image (larger images read them from L2)
  static constexpr bool W1X_LDS = !BLOCKED && !BWD && NMAX <= 32;
  alignas(16) float w1x[W1X_LDS ? NT * KS0MAX * 512 : 4];
  alignas(16) float agg[RB * AST];
  alignas(16) float head[BWD ? 1 : WAVES][BWD ? 1 : H + 4];
  uint32_t pairs[PC];
  uint32_t mask27[NMAX];
  // <= 32-atom images: the surviving periodic images that can reach the
  // molecule's bounding box within r_cut (bit s of near27[a]), their positions
  // imgp[a][s] kept in the edge_nn.0 fragment buffer (free during the pair build)
  static constexpr bool IMG_LDS = W1X_LDS && NT * KS0MAX * 512 >= NMAX * 27 * 4;
  uint32_t near27[IMG_LDS ? NMAX : 1];
  float bbox[8];
  int idmap[NMAX];
  int cntrow[NMAX];
  int headrow[WAVES];
  int ishead[WAVES];
  int scan[WAVES];
  int npairs;                         // pairs in the buffer (this pass)
  int ptotal;                         // pairs of the whole block
  int err;
  uint32_t big;                       // BIGK_* seen this layer / row block (F16X3 small-operand guard)
  float red[WAVES];
  static constexpr int NDT = BWD ? 1 : NT, NDR = BWD ? 1 : RB;
  // <= 32-atom images (and the large-system row blocks): the edge tiles' message
  // segment sums go through a per-wave LDS scratch [32 pairs][MSP] in the union
  // (free during the tiles); other images scan in registers (seg_scan4x)
  static constexpr bool MSG_LDS = ENFLOW_MSG_LDS && !BWD && NMAX == 32 && RB == 32;
  static constexpr int MSW = H < 64 ? H : 64;                         // features per reduce chunk
  static constexpr int MSP = MSW + 1;                                 // odd row stride: conflict-free
  // <= 32-atom images, split precision: the message segment sums run on the
  // matrix cores (edge_tiles): per wave the fp16 hi | lo image of one 32-feature
  // tile of the messages, [32 pairs][34 dwords] (136-B rows: the pair-lane
  // stores are 2-way, the transposed reads of 4 rows at most 2-way), the pair
  // tile's selection words (f16 multiplicity << 16 | segment) and segment rows
  static constexpr bool MSG_MMA = ENFLOW_MSG_MFMA && !MSG_LDS && !BWD && NMAX == 32 && RB == 32;
  static constexpr int MIS = 34;
  union {
    int C[CW];                                                    // pair build (block rows x atoms)
    float msg[MSG_LDS ? WAVES : 1][MSG_LDS ? 32 * MSP : 1];       // edge tiles: per-wave message scratch
    struct {
      alignas(16) uint32_t img[MSG_MMA ? WAVES : 1][MSG_MMA ? 32 * MIS : 1];
      alignas(16) uint32_t tb[MSG_MMA ? WAVES : 1][32];
      int rt[MSG_MMA ? WAVES : 1][32];
    } mm;                                                         // edge tiles: message MFMA operands
    struct { float qp[NDT][NDR]; float gp[NDT][NFMAX][NDR]; } nd;   // node phase partials
    float net[NETA * 2 * NFMAX];                                  // ArgMax outputs
    float nb[NBW];                                                // BWD: node adjoint rows
  } u;
};

// multiplicity count e of the block (int, or packed 16-bit when blocked: a count
// is at most 27 images x 27 repeated labels < 2^16)
template <class S>
__device__ __forceinline__ int c_get(const S& sm, int e) {
  if constexpr (S::PACKC) return (sm.u.C[e >> 1] >> (16 * (e & 1))) & 0xffff;
  else return sm.u.C[e];
}
template <class S>
__device__ __forceinline__ void c_add(S& sm, int e, int v) {
  if constexpr (S::PACKC) atomicAdd(&sm.u.C[e >> 1], v << (16 * (e & 1)));
  else atomicAdd(&sm.u.C[e], v);
}

struct MolRef {
  int a0, n;
  float rc;
  float bx, by, bz;   // the molecule's edge box = box of its first atom (base.py:130)
  int m = 0;          // molecule index in the batch (FlowArgs::mol_list may map blocks to molecules)
};

// ---------------------------------------------------------------------------
// neighbour list: Data.edges (enflow/data/base.py:122-144) for one molecule
// ---------------------------------------------------------------------------
__device__ __forceinline__ float shift_of(int idx, float b) { return idx == 0 ? -b : (idx == 1 ? b : 0.f); }

// (a) image masks and (b) id_mapping for all atoms of the molecule (once per layer)
template <class S>
__device__ __forceinline__ void build_images(S& sm, const MolRef& M, int tid) {
  const int n = M.n;
  const float rx = M.bx + M.rc, ry = M.by + M.rc, rz = M.bz + M.rc;   // helpers.py:20
  for (int a = tid; a < n; a += BLOCK) {
    sm.mask27[a] = 0u;
    sm.idmap[a] = -1;
    sm.cntrow[a] = 0;
    if constexpr (S::IMG_LDS) sm.near27[a] = 0u;
  }
  if constexpr (!S::BLOCKED) {   // the whole molecule's count matrix, zeroed here: block_counts(.., zeroed)
    const int words = S::PACKC ? (n * n + 1) / 2 : n * n;
    for (int e = tid; e < words; e += BLOCK) sm.u.C[e] = 0;
  }
  if constexpr (S::IMG_LDS) {   // the molecule's bounding box (n <= 32: one wave)
    if (tid < 64) {
      float lo[3], hi[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const float x = tid < n ? sm.pos[tid * 3 + d] : sm.pos[d];
        hi[d] = wave_max(x);
        lo[d] = -wave_max(-x);
      }
      if (tid < 3) {
        sm.bbox[tid] = tid == 0 ? lo[0] : (tid == 1 ? lo[1] : lo[2]);
        sm.bbox[4 + tid] = tid == 0 ? hi[0] : (tid == 1 ? hi[1] : hi[2]);
      }
    }
  }
  __syncthreads();
  // (a) image masks, one (atom, image) per thread: bit s <=> image s of atom a
  //     lies in the ellipsoid with radii box + r_cut (helpers.py:17-22)
  const float r_sq = M.rc * M.rc;
  //     one (atom, y/z shift) per thread, its three x shifts in registers
  for (int e = tid; e < n * 9; e += BLOCK) {
    const int a = e / 9, yz = e - a * 9;
    const float iy = sm.pos[a * 3 + 1] + shift_of(yz % 3, M.by);
    const float iz = sm.pos[a * 3 + 2] + shift_of(yz / 3, M.bz);
    const float sy = iy / ry, sz = iz / rz;
    float ey = 0.f, ez = 0.f;
    if constexpr (S::IMG_LDS) {
      ey = fmaxf(fmaxf(sm.bbox[1] - iy, iy - sm.bbox[5]), 0.f);
      ez = fmaxf(fmaxf(sm.bbox[2] - iz, iz - sm.bbox[6]), 0.f);
    }
    uint32_t mk = 0u, nr = 0u;
#pragma unroll
    for (int xs = 0; xs < 3; ++xs) {
      const int s = xs + 3 * yz;
      const float ix = sm.pos[a * 3 + 0] + shift_of(xs, M.bx);
      const float sx = ix / rx;
      if (sx * sx + sy * sy + sz * sz <= 1.0f) {
        mk |= 1u << s;
        if constexpr (S::IMG_LDS) {
          // farther than r_cut from the bounding box (1e-4 relative margin over fp32
          // rounding) no atom can be hit: the image is skipped by the distance tests
          const float ex = fmaxf(fmaxf(sm.bbox[0] - ix, ix - sm.bbox[4]), 0.f);
          if (ex * ex + ey * ey + ez * ez <= r_sq * 1.0001f) {
            nr |= 1u << s;
            st4(&sm.w1x[(a * 27 + s) * 4], (f32x4){ix, iy, iz, 0.f});
          }
        }
      }
    }
    if (mk) atomicOr(&sm.mask27[a], mk);
    if constexpr (S::IMG_LDS) {
      if (nr) atomicOr(&sm.near27[a], nr);
    }
  }
  __syncthreads();
  // (b) id_mapping[q] for q < n: the q-th surviving image in (image, atom) order (helpers.py:25-27)
  if (tid < 64) {
    const int lane = tid;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int prefix = 0;
    if (n <= 64) {   // one chunk: the lane's mask loaded once, 27 ballots on registers
      const uint32_t mk = lane < n ? sm.mask27[lane] : 0u;
      for (int s = 0; s < 27 && prefix < n; ++s) {
        const bool bit = (mk >> s) & 1u;
        const uint64_t bal = __ballot(bit);
        if (bit) {
          const int posF = prefix + __popcll(bal & lt);
          if (posF < n) sm.idmap[posF] = lane;
        }
        prefix += __popcll(bal);
      }
    } else {
      for (int s = 0; s < 27 && prefix < n; ++s) {
        for (int ch = 0; ch < n; ch += 64) {
          const int a = ch + lane;
          const uint32_t mk = a < n ? sm.mask27[a] : 0u;
          const bool bit = (mk >> s) & 1u;
          const uint64_t bal = __ballot(bit);
          if (bit) {
            const int posF = prefix + __popcll(bal & lt);
            if (posF < n) sm.idmap[posF] = a;
          }
          prefix += __popcll(bal);
        }
      }
    }
    // prefix < n: atom columns q >= prefix have no id_mapping entry (idmap -1);
    // the reference raises only if such a column has a hit (block_counts)
  }
  __syncthreads();
}

// (c) multiplicity matrix of rows r0 .. r0 + rb - 1: C[i][id_mapping[q]] += #images
//     of i within r_cut of atom q (base.py:133-139: both hit columns mapped through
//     id_mapping, self pairs dropped), (d) compaction to (local row, col, mult)
//     sorted by (row, col).
template <class S>
__device__ __forceinline__ void block_counts(S& sm, const MolRef& M, int tid, int r0, int rb, bool zeroed = false) {
  const int n = M.n;
  if (!zeroed) {   // (build_images zeroes the whole molecule's matrix before its barriers)
    const int words = S::PACKC ? (rb * n + 1) / 2 : rb * n;
    for (int e = tid; e < words; e += BLOCK) sm.u.C[e] = 0;
    __syncthreads();
  }
  const float r_sq = M.rc * M.rc;
  for (int e = tid; e < rb * n; e += BLOCK) {
    const int il = e / n, q = e - il * n;
    const int i = r0 + il;
    const int jl = sm.idmap[q];
    if (jl == i) continue;             // self pair by label (base.py:139)
    const float qx = sm.pos[q * 3 + 0], qy = sm.pos[q * 3 + 1], qz = sm.pos[q * 3 + 2];
    int cnt = 0;
    if constexpr (S::IMG_LDS) {   // the row's near images, positions precomputed (same fp32 values)
      uint32_t bits = sm.near27[i];
      const float* img = &sm.w1x[i * 27 * 4];
      while (bits) {
        const int s = __builtin_ctz(bits);
        bits &= bits - 1;
        const f32x4 im = ld4(img + 4 * s);
        const float dx = im[0] - qx, dy = im[1] - qy, dz = im[2] - qz;
        if (dx * dx + dy * dy + dz * dz < r_sq) ++cnt;
      }
    } else {
      const float px = sm.pos[i * 3 + 0], py = sm.pos[i * 3 + 1], pz = sm.pos[i * 3 + 2];
      uint32_t bits = sm.mask27[i];
      while (bits) {
        const int s = __builtin_ctz(bits);
        bits &= bits - 1;
        const float ix = px + shift_of(s % 3, M.bx), iy = py + shift_of((s / 3) % 3, M.by),
                    iz = pz + shift_of(s / 9, M.bz);
        const float dx = ix - qx, dy = iy - qy, dz = iz - qz;
        if (dx * dx + dy * dy + dz * dz < r_sq) ++cnt;
      }
    }
    if (cnt) {
      if (jl < 0) {                    // a hit on column q past id_mapping: the reference's
        sm.err |= ENFLOW_ERR_FEW_IMAGES;   // IndexError (base.py:137)
        continue;
      }
      c_add(sm, il * n + jl, cnt);
      atomicAdd(&sm.cntrow[i], cnt);
    }
  }
  __syncthreads();
}

// (d) compaction of the block's counts to (local row, col, mult) sorted by
// (row, col): the pairs of rank p0 .. p0 + PC - 1 go to the pair buffer
// (sm.npairs of them); returns the block's total (sm.ptotal).
template <class S>
__device__ __forceinline__ int block_compact(S& sm, int n, int tid, int rb, int p0) {
  constexpr int PC = S::PC;
  const int NN = rb * n;
  const int per = (NN + BLOCK - 1) / BLOCK;
  const int e0 = tid * per, e1 = min(NN, e0 + per);
  int local = 0;
  for (int e = e0; e < e1; ++e) local += c_get(sm, e) > 0;
  const int incl = wave_incl_scan(local);
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave index: SGPR
  if (lane == 63) sm.scan[w] = incl;
  __syncthreads();
  int base = incl - local;
  for (int k = 0; k < w; ++k) base += sm.scan[k];
  for (int e = e0; e < e1; ++e) {
    const int c = c_get(sm, e);
    if (c > 0) {
      if (base >= p0 && base < p0 + PC) {
        const int il = e / n, jl = e - il * n;
        sm.pairs[base - p0] = (uint32_t)il | ((uint32_t)jl << 8) | ((uint32_t)c << 16);
      }
      ++base;
    }
  }
  if (tid == BLOCK - 1) {
    int tot = 0;
    for (int k = 0; k < WAVES; ++k) tot += sm.scan[k];
    sm.ptotal = tot;
    sm.npairs = min(tot - p0, PC);
  }
  __syncthreads();
  return sm.ptotal;
}

template <class S>
__device__ __forceinline__ void build_block_pairs(S& sm, const MolRef& M, int tid, int r0, int rb) {
  static_assert(!S::BLOCKED, "blocked images compact in passes (block_compact)");
  block_counts(sm, M, tid, r0, rb, r0 == 0 && rb == M.n);   // after build_images: already zeroed
  block_compact(sm, M.n, tid, rb, 0);
}

// whole-molecule pair list (one block)
template <class S>
__device__ __forceinline__ void build_pairs(S& sm, const MolRef& M, int tid) {
  static_assert(!S::BLOCKED, "build_pairs needs the unblocked image");
  build_images(sm, M, tid);
  build_block_pairs(sm, M, tid, 0, M.n);
}

// ---------------------------------------------------------------------------
// EGCL edge part: per-pair MLP chain on MFMA + deterministic segment sums
// ---------------------------------------------------------------------------
//
// BIG (large-system path, enflow_large.hip): the image holds only the block's
// rows; pair words are (row | col << 5 | mult << 27) and the column atoms'
// positions / features are read from global memory (cpos / ch, molecule-local
// rows, L2-resident).
template <bool BIG>
__device__ __forceinline__ int pair_row(uint32_t pr) { return BIG ? (int)(pr & 31u) : (int)(pr & 0xffu); }

// pre(): run by every wave after its last tile, before the closing barrier (the
// node phase's fragment requests, so their L2 round trip overlaps the wait)
template <int H, int NMAX, int RB, int PREC = PREC_F32, bool VAR = false, bool BIG = false, class Pre = NoMid>
__device__ __forceinline__ void edge_tiles(Smem<H, NMAX, RB>& sm, const float* __restrict__ Lp, const EgclLayout& L,
                                           const MolRef& M, int nf, int tid, int r0, int rb,
                                           bool zero_agg STAMP_ARGS, const float* __restrict__ cpos = nullptr,
                                           const float* __restrict__ ch = nullptr, Pre&& pre = NoMid{}) {
  constexpr int NT = H / 32;
  constexpr int AST = Smem<H, NMAX, RB>::AST;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave index: SGPR
  const int j = lane & 31, hh = lane >> 5;
  const int P = sm.npairs;
  const int T = (P + 31) >> 5;
  const int tpw = (T + WAVES - 1) / WAVES;

  // zero aggregates / heads, stage biases, find each wave's head row
  if (zero_agg)   // first compaction pass of the block (later passes accumulate)
    for (int e = tid; e < rb * AST; e += BLOCK) sm.agg[e] = 0.f;
  for (int e = tid; e < WAVES * (H + 4); e += BLOCK) (&sm.head[0][0])[e] = 0.f;
  // split-precision GEMMs run on weights scaled by 2^s (K below): the bias image
  // carries the same factor, the accumulators start from it (acc_from_bias)
  const float K0 = PREC != PREC_F32 ? Lp[L.scl + 4] : 1.f;   // edge_nn.0 runs F16X3 in bf16 mode too
  const float K1 = PREC == PREC_F16X3 ? Lp[L.scl + 0] : 1.f;
  const float K2 = PREC == PREC_F16X3 ? Lp[L.scl + 2] : 1.f;
  for (int k = tid; k < H; k += BLOCK) {
    sm.bias[k] = Lp[L.be1 + k] * K0;
    sm.bias[H + k] = Lp[L.be2 + k] * K1;
    sm.bias[2 * H + k] = Lp[L.bc1 + k] * K2;
    sm.bias[3 * H + k] = Lp[L.wc2 + k];
  }
  if constexpr (PREC != PREC_F32 && Smem<H, NMAX, RB>::W1X_LDS) {   // GEMM0 is F16X3 in bf16 mode too
    // edge_nn.0 split fragments: one L2 pass per layer instead of one per tile
    const int ks_n = gemm0_ksteps(nf);
    for (int e = tid; e < NT * ks_n * 128; e += BLOCK) {   // 128 x 16 B per (t, ks)
      const int blk = e >> 7, r = e & 127, ln = r >> 1, part = r & 1;
      const int t = blk / ks_n, ks = blk - t * ks_n;
      const f32x4 v = ld4(Lp + L.we1x + (t * KS0MAX + ks) * 512 + ln * 8 + part * 4);
      st4(&sm.w1x[(t * KS0MAX + ks) * 512 + part * 256 + ln * 4], v);
    }
  }
  if (tid < WAVES) {
    const int t0 = tid * tpw;
    int hr = -1, ih = 0;
    if (t0 < T) {
      const int p0 = t0 * 32;
      hr = pair_row<BIG>(sm.pairs[p0]);
      ih = (p0 > 0) && (pair_row<BIG>(sm.pairs[p0 - 1]) == hr);
    }
    sm.headrow[tid] = hr;
    sm.ishead[tid] = ih;
  }
  __syncthreads();

  const int t0 = w * tpw, t1 = min(T, t0 + tpw);
  const int headrow = sm.headrow[w];
  const bool ishead = sm.ishead[w] != 0;
  const int nh = (nf + 1) >> 1;
  const rsrc_t W = weights_rsrc(Lp, L.total);
  const float hbx = M.bx * 0.5f, hby = M.by * 0.5f, hbz = M.bz * 0.5f;
  // scaled SiLU constants (silu4s): c = -log2(e) / K
  constexpr float NLOG2E = -1.4426950408889634f;
  const float ik0 = PREC != PREC_F32 ? Lp[L.scl + 5] : 1.f;   // 1 / K0 .. 1 / K2 (exact powers of two)
  const float ik1 = PREC == PREC_F16X3 ? Lp[L.scl + 1] : 1.f;
  const float ik2 = PREC == PREC_F16X3 ? Lp[L.scl + 3] : 1.f;
  const float c0 = NLOG2E * ik0, c1 = NLOG2E * ik1, c2 = NLOG2E * ik2;
  constexpr bool MSG_LDS = Smem<H, NMAX, RB>::MSG_LDS;
  // VAR: +0.8 KB scratch; BIG (enflow_large.hip's row blocks): +0.6 KB scratch, 3x slower
  constexpr bool MMA = PREC != PREC_F32 && !VAR && !BIG && Smem<H, NMAX, RB>::MSG_MMA;
  // weight-fragment ring depth of GEMM1 / GEMM2 (the headline instance: 3)
  constexpr int XD = (NMAX == 32 && RB == 32 && WAVES == 4 && !BIG) ? ENFLOW_FWD_X3_DEPTH : ENFLOW_X3_DEPTH;
  constexpr int MIS = Smem<H, NMAX, RB>::MIS;
  constexpr int MSP = Smem<H, NMAX, RB>::MSP;
  float* const scr = MSG_LDS ? &sm.u.msg[w][0] : nullptr;
  // constructor variants of the layer (wave-uniform; compiled in only for VAR
  // kernels, the default-flag kernels keep their registers)
  const int vfl = VAR ? (int)Lp[L.vfl] : 0;
  const bool v_att = (vfl & EGCL_ATTENTION) != 0, v_nd = (vfl & EGCL_NORM_DIFF) != 0,
             v_tanh = (vfl & EGCL_TANH) != 0;
  const Act act = VAR ? act_of(Lp + L.vfl + 1) : act_silu();   // act_fn (egcl.py:11)

  // split-precision range check: an fp16 / bf16 operand past its range makes the
  // MFMA products inf / NaN; the per-pair scalars where the reference's own ops
  // would squash that back to a finite value (tanh, the clamp, the attention
  // sigmoid) are tested here, everything else propagates to the outputs, which
  // the kernels test as well (ENFLOW_ERR_RANGE)
  bool range_bad = false;
  constexpr bool GUARD = PREC == PREC_F16X3;   // small-operand guard (BIGK_*)
  uint32_t bigw = 0u;                          // wave-uniform
  STAMP(8);
  for (int tile = t0; tile < t1; ++tile) {
    const int p = tile * 32 + j;
    const bool valid = p < P;
    uint32_t o0 = 0u, o1 = 0u, o2 = 0u;   // OR of the operands' packed fp16 hi words
    const uint32_t vmask = valid ? ENFLOW_BIG_BITS : 0u;   // padding lanes (row 0's atoms) do not count
    // each kind's word is tested right after its GEMM (one VGPR live through one chain)
    auto seen_big = [&](uint32_t o, uint32_t kind) {
      if constexpr (GUARD) bigw |= __ballot((o & vmask) != 0u) ? kind : 0u;
    };
    const uint32_t pr = valid ? sm.pairs[p] : 0u;
    const int il = pair_row<BIG>(pr);
    const int jl = BIG ? (int)((pr >> 5) & 0x3fffffu) : (int)((pr >> 8) & 0xffu);
    const int i = r0 + il;                 // atom of the row (il: row within the block)
    const float c = (float)(BIG ? (pr >> 27) : (pr >> 16));
    // column atom's coordinates / features: LDS image, or global (BIG)
    auto cp = [&](int d) {
      if constexpr (BIG) return cpos[(size_t)jl * 3 + d];
      else return sm.pos[jl * 3 + d];
    };
    auto chf = [&](int k) {   // k < nf
      if constexpr (BIG) return ch[(size_t)jl * nf + k];
      else return sm.h[jl * NFP + k];
    };
    // segments = runs of equal row; invalid lanes get unique rows of their own
    const int row = valid ? il : -1 - j;
    // segment masks: the exact (EXEC) form for the forces -- phi feeds the
    // clamp, whose NaN must stay NaN -- and the multiplier form for the message
    // scans (1 VALU per value and step; its 0 * NaN can spread a NaN input to a
    // neighbouring row of the same molecule, never turn it finite)
    const SegExec SE = seg_exec(row);
    SegMasks SM;
    if constexpr (!MSG_LDS && !MMA) SM = seg_masks(row);
    int nseg = 0;
    if constexpr (MMA) {
      // the tile's segments: slot = index of the row run (invalid lanes are runs
      // of their own with multiplicity 0); the selection word of pair j and the
      // row of every slot go to the wave's tables, read back by segment lanes
      const int row_prev = __shfl_up(row, 1, 32);
      const bool start = j == 0 || row_prev != row;
      const uint32_t S = (uint32_t)__ballot(start);
      const int seg = __builtin_popcount(S & (uint32_t)((2ull << j) - 1ull)) - 1;
      nseg = __builtin_popcount(S);
      if (hh == 0) {
        sm.u.mm.tb[w][j] = ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)c) << 16) | (uint32_t)seg;
        if (start) sm.u.mm.rt[w][seg] = valid ? il : -1;
      }
    }
    const int row_next = __shfl_down(row, 1, 32);
    const bool seg_end = valid && (j == 31 || row_next != row);
    float* const dst_row = (ishead && row == headrow) ? &sm.head[w][0] : &sm.agg[(valid ? il : 0) * AST];
    // Edges.coord_diff with the reference's half-box image (base.py:15-19)
    const float dx = pbc1(sm.pos[i * 3 + 0] - cp(0), hbx);
    const float dy = pbc1(sm.pos[i * 3 + 1] - cp(1), hby);
    const float dz = pbc1(sm.pos[i * 3 + 2] - cp(2), hbz);
    const float radial = dx * dx + dy * dy + dz * dz;                 // egcl.py:79

    // GEMM1's first fragments requested now: their L2 round trip overlaps GEMM0
    X3Ring<NT, XD> ring1;
    if constexpr (PREC == PREC_F16X3) x3_prologue(ring1, W, L.we2x, lane);
    // ---- GEMM0: X0^T = edge_nn.0.weight . [h_i, h_j, radial]^T  (egcl.py:57-58)
    //      9 fixed k-steps (zero-padded past nf): 4 h_i pairs, 4 h_j pairs, radial;
    //      h rows are zero-padded in LDS, so padded steps multiply zeros
    f32x16 x0[NT];
    acc_from_bias<NT>(x0, sm.bias, hh);
    if constexpr (PREC != PREC_F32) {   // F16X3 (bf16 mode too: a 16-wide k-step on the matrix cores
      // beats 9 f32 k-steps; only edge_nn.2 / coord_nn.0 run in bf16)
      // k order gemm0_col: lane half 0 = h_i's padded row, half 1 = h_j's (+ radial)
      const int ks_n = gemm0_ksteps(nf), nch = gemm0_nch(nf);
      for (int ks = 0; ks < ks_n; ++ks) {
        f32x16 in;
        if (ks < nch) {
          const int f0 = 8 * ks;
          if constexpr (BIG) {
#pragma unroll
            for (int jj = 0; jj < 8; ++jj)
              in[jj] = hh ? (f0 + jj < nf ? chf(f0 + jj) : 0.f) : sm.h[i * NFP + f0 + jj];
          } else {
            const float* hrow = &sm.h[(hh ? jl : i) * NFP + f0];   // rows zero-padded past nf
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) in[jj] = hrow[jj];
          }
          if (hh && ks == nch - 1 && gemm0_radial_slot7(nf)) in[7] = radial;
        } else {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) in[jj] = 0.f;
          if (hh == 0) in[0] = radial;
        }
        f16x8 bh, bl;
        split_f16(in, 0, bh, bl);
        if constexpr (GUARD) o0 = or_hi(o0, bh);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          f32x4 ah, al;
          if constexpr (Smem<H, NMAX, RB>::W1X_LDS) {
            ah = ld4(&sm.w1x[(t * KS0MAX + ks) * 512 + lane * 4]);
            al = ld4(&sm.w1x[(t * KS0MAX + ks) * 512 + 256 + lane * 4]);
          } else {
            const int so = (L.we1x + (t * KS0MAX + ks) * 512) * 4;
            ah = bload4(W, lane * 32, so);
            al = bload4(W, lane * 32 + 16, so);
          }
          x0[t] = mfma_f16(ah, bh, x0[t]);
          x0[t] = mfma_f16(ah, bl, x0[t]);
          x0[t] = mfma_f16(al, bh, x0[t]);
        }
      }
    } else {
      float cur[NT], nxt[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) cur[t] = bload(W, lane * 4, (L.we1f + (t * (NFMAX + 1)) * 64) * 4);
#pragma unroll
      for (int s = 0; s < NFMAX + 1; ++s) {
        if (s + 1 < NFMAX + 1) {
#pragma unroll
          for (int t = 0; t < NT; ++t) nxt[t] = bload(W, lane * 4, (L.we1f + (t * (NFMAX + 1) + s + 1) * 64) * 4);
        }
        float hj;
        if constexpr (BIG) {   // global rows are not zero-padded past nf
          const int kj = 2 * (s - NFMAX / 2) + hh;
          hj = (s >= NFMAX / 2 && s < NFMAX && kj < nf) ? chf(kj) : 0.f;
        } else {
          hj = (s >= NFMAX / 2 && s < NFMAX) ? sm.h[jl * NFP + 2 * (s - NFMAX / 2) + hh] : 0.f;
        }
        const float b = s < NFMAX / 2 ? sm.h[i * NFP + 2 * s + hh] : (s < NFMAX ? hj : (hh == 0 ? radial : 0.f));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < NT; ++t) x0[t] = mfma32(cur[t], b, x0[t]);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < NFMAX + 1) {
#pragma unroll
          for (int t = 0; t < NT; ++t) cur[t] = nxt[t];
        }
      }
    }
    STAMP(9);
    seen_big(o0, BIGK_X0);
    // x0 tile 0 activated now, tiles 1.. as fillers of GEMM1's steps on tile t-1
    // (split-precision GEMM0 accumulators carry edge_nn.0's 2^s: unscaled in the bias fma)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 y = act4s<VAR>((f32x4){x0[0][4 * g4], x0[0][4 * g4 + 1], x0[0][4 * g4 + 2], x0[0][4 * g4 + 3]},
                                 c0, K0, ik0, act);
#pragma unroll
      for (int u = 0; u < 4; ++u) x0[0][4 * g4 + u] = y[u];
    }
    STAMP(10);

    // ---- GEMM1: E^T = edge_nn.2 (egcl.py:20-24)
    f32x16 e[NT];
    acc_from_bias<NT>(e, sm.bias + H, hh);
    auto fill1 = [&](int step) {
      const int t = (step >> 2) + 1, g4 = step & 3;
      if (t < NT) {
        const f32x4 y = act4s<VAR>((f32x4){x0[t][4 * g4], x0[t][4 * g4 + 1], x0[t][4 * g4 + 2], x0[t][4 * g4 + 3]},
                                   c0, K0, ik0, act);
#pragma unroll
        for (int u = 0; u < 4; ++u) x0[t][4 * g4 + u] = y[u];
      }
    };
    if constexpr (PREC == PREC_F16X3)
      chain_x3_fill_r<NT, ENFLOW_FPM1, XD>(W, L.we2x, x0, e, lane, ring1, fill1, NoMid{}, NoLate{},
                                           [&](int, const f16x8& bh, const f16x8&) { o1 = or_hi(o1, bh); });
    else chain_prec_fill<PREC, NT, ENFLOW_FPM1, XD>(W, L.we2f, L.we2x, L.we2b, x0, e, lane, fill1);
    seen_big(o1, BIGK_Y0);
    // GEMM2's first fragments (the message-MFMA path) requested before e's activation
    X3Ring<NT, XD> ring2;
    if constexpr (PREC == PREC_F16X3 && MMA) x3_prologue(ring2, W, L.wc1x, lane);
    STAMP(11);
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 y = act4s<VAR>((f32x4){e[0][4 * g4], e[0][4 * g4 + 1], e[0][4 * g4 + 2], e[0][4 * g4 + 3]},
                                 c1, K1, ik1, act);
#pragma unroll
      for (int u = 0; u < 4; ++u) e[0][4 * g4 + u] = y[u];
    }
    if (v_att) {   // egcl.py:60-62: out *= sigmoid(att_nn(out)); every tile activated first
#pragma unroll
      for (int t = 1; t < NT; ++t)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
          for (int u = 0; u < 4; ++u) e[t][4 * g4 + u] = act_sc<VAR>(e[t][4 * g4 + u], c1, K1, ik1, act);
      float d = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 wa = ld4(Lp + L.watt + 32 * t + 8 * g4 + 4 * hh);
#pragma unroll
          for (int u = 0; u < 4; ++u) d = fmaf(wa[u], e[t][4 * g4 + u], d);
        }
      const float dl = d + __shfl_xor(d, 32, 64) + Lp[L.batt];
      if constexpr (PREC != PREC_F32) range_bad |= valid && !__builtin_isfinite(dl);
      const float att = sigm_f(dl);
#pragma unroll
      for (int t = 0; t < NT; ++t) e[t] *= att;
    }
    STAMP(12);
    STAMP(13);
    // ---- GEMM2: coord_nn.0 (egcl.py:35-42), with fillers: activate e tile t+1
    //      and segment-sum the messages of tile t (egcl.py:64-65, multiplicity-
    //      weighted, DPP segmented scan; the row's last lane adds its 4 features
    //      into the row with one ds_read_b128 / ds_write_b128 at a constant offset:
    //      the read is issued before the scan (every lane reads its own row, only
    //      segment ends write), one adder per (row, feature) and tile)
    float* const rowp = dst_row + 4 * hh;
    float part = 0.f;
    // message segment sums, LDS images: c e[t] of feature tile t goes to the wave's
    // scratch (row = pair, 64-feature chunks); a chunk is reduced by feature lanes
    // walking the tile's 32 pairs in order and adding each finished row segment
    // into its aggregate row (uniform control: the segment ends are one mask)
    const uint32_t endm = (uint32_t)__ballot(seg_end && hh == 0);
    auto reduce_chunk = [&](int chn) {
      if constexpr (MSG_LDS) {
        const int f = lane;                        // feature (MSP - 1) chn + lane of the chunk
        const bool fv = lane < MSP - 1;            // H = 32: 32 features, lanes 32.. idle
        const float* col = scr + (fv ? f : 0);
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < 32; ++q) {
          acc += col[q * MSP];
          if (endm & (1u << q)) {
            const int r = __builtin_amdgcn_readlane(row, q);
            float* d = (ishead && r == headrow) ? &sm.head[w][0] : &sm.agg[r * AST];
            if (fv) atomicAdd(d + (MSP - 1) * chn + f, acc);   // one wave adds to a row: fixed order
            acc = 0.f;
          }
        }
      }
    };
    if constexpr (MMA) {
      // message segment sums on the matrix cores: agg[row(n)][f] += sum_p
      // E[p][f] S[p][n], S[p][n] = c_p if pair p is in segment n -- one
      // 32x32x16 MFMA per (32-feature tile, 16 pairs, hi | lo) with A = E^T
      // (features x pairs) read transposed from the fp16 image that GEMM2's own
      // operand split writes, B = S (pairs x segment slots).  The accumulator
      // starts from the segment rows' aggregates and is stored back by the
      // lanes of the tile's segments (lane = slot n: features 8 g4 + 4 hh + u).
      f32x16 hc[NT];
      acc_from_bias<NT>(hc, sm.bias + 2 * H, hh);
      uint32_t* const img = &sm.u.mm.img[w][0];
      const int ibase = (8 * hh + ((lane >> 2) & 3)) * MIS + 2 * (4 * ((lane >> 4) & 1) + (lane & 3));
      f16x8 sel[2];
      float* dstn = &sm.agg[0];
      bool vn = false;
      f32x16 Y;
      s16x4 ar[4][2];
      u32x4v tq[4];
      int rn = -1;
      // LDS reads are issued MSTEP chain steps (their MFMAs) before their use.
      // Feature tile t's image is complete after k-slice 2 t + 1's split, at
      // step (2 t + 1) AB - 1, and k-slice 2 t + 2 overwrites it at the end of
      // step (2 t + 2) AB - 1 (AB = chain steps per k-slice)
      constexpr int AB = PREC == PREC_F16X3 ? NT : 1;
      constexpr int MSTEP = AB >= 4 ? 2 : 1;   // tile reads at step a, MFMAs at a + MSTEP, stores after
      auto late = [&](int step) {
        if (step == 0) {
          const uint32_t* const tb = &sm.u.mm.tb[w][0];
#pragma unroll
          for (int q = 0; q < 4; ++q) tq[q] = *reinterpret_cast<const u32x4v*>(tb + 16 * (q >> 1) + 8 * hh + 4 * (q & 1));
          rn = sm.u.mm.rt[w][j];
        }
        if (step == 1) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const u32x4v q0 = tq[2 * ks], q1 = tq[2 * ks + 1];
            const uint32_t wv[8] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3]};
            u32x4v pk;
#pragma unroll
            for (int i2 = 0; i2 < 4; ++i2) {
              const uint32_t a0 = (wv[2 * i2] & 0xffffu) == (uint32_t)j ? wv[2 * i2] >> 16 : 0u;
              const uint32_t a1 = (wv[2 * i2 + 1] & 0xffffu) == (uint32_t)j ? wv[2 * i2 + 1] & 0xffff0000u : 0u;
              pk[i2] = a0 | a1;
            }
            sel[ks] = __builtin_bit_cast(f16x8, pk);
          }
          vn = j < nseg && rn >= 0;
          if (vn) dstn = (ishead && rn == headrow) ? &sm.head[w][0] : &sm.agg[rn * AST];
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int a = (2 * t + 1) * AB;
          if (step == a) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
              for (int rd = 0; rd < 2; ++rd) ar[k][rd] = lds_tr16(img + ibase + (16 * (k >> 1) + 4 * rd) * MIS + 16 * (k & 1));
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
              const f32x4 v = ld4(dstn + 32 * t + 8 * g4 + 4 * hh);
#pragma unroll
              for (int u = 0; u < 4; ++u) Y[4 * g4 + u] = v[u];
            }
          }
          if (step == a + MSTEP) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(cat_f16x8(ar[k][0], ar[k][1]), sel[k >> 1], Y, 0, 0, 0);
          }
          if (step == a + MSTEP + 1 && vn) {
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) st4(dstn + 32 * t + 8 * g4 + 4 * hh, (f32x4){Y[4 * g4], Y[4 * g4 + 1],
                                                                                     Y[4 * g4 + 2], Y[4 * g4 + 3]});
          }
        }
      };
      auto onsplit = [&](int ts, const f16x8& bh, const f16x8& bl) {
        if constexpr (GUARD) o2 = or_hi(o2, bh);
        const u32x4v hv = __builtin_bit_cast(u32x4v, bh), lv = __builtin_bit_cast(u32x4v, bl);
        uint32_t* const r = img + j * MIS + 2 * hh + 8 * (ts & 1);   // 4-feature unit 4 s + hh (+2, +8: lo)
        *reinterpret_cast<u32x2v*>(r) = (u32x2v){hv[0], hv[1]};
        *reinterpret_cast<u32x2v*>(r + 4) = (u32x2v){hv[2], hv[3]};
        *reinterpret_cast<u32x2v*>(r + 16) = (u32x2v){lv[0], lv[1]};
        *reinterpret_cast<u32x2v*>(r + 20) = (u32x2v){lv[2], lv[3]};
      };
      auto fillm = [&](int step) {
        const int t = step >> 2, g4 = step & 3;
        if (t + 1 < NT && !v_att) {
          const f32x4 y = act4s<VAR>((f32x4){e[t + 1][4 * g4], e[t + 1][4 * g4 + 1], e[t + 1][4 * g4 + 2],
                                             e[t + 1][4 * g4 + 3]}, c1, K1, ik1, act);
#pragma unroll
          for (int u = 0; u < 4; ++u) e[t + 1][4 * g4 + u] = y[u];
        }
      };
      if constexpr (PREC == PREC_F16X3) {
        chain_x3_fill_r<NT, ENFLOW_FPM2, XD>(W, L.wc1x, e, hc, lane, ring2, fillm, NoMid{}, late, onsplit);
      } else {   // bf16 GEMM2: the image gets an fp16 hi / lo split of its own
        chain_b16_fill<NT, ENFLOW_FPM2>(W, L.wc1b, e, hc, lane, fillm, NoMid{}, late, [&](int ts) {
          f16x8 bh, bl;
          split_f16(e[ts >> 1], ts & 1, bh, bl);
          onsplit(ts, bh, bl);
        });
      }
      seen_big(o2, BIGK_M);
      // coord_nn.2 as a per-pair dot
#pragma unroll
      for (int tp = 0; tp < NT; ++tp)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 w2 = *reinterpret_cast<const f32x4*>(sm.bias + 3 * H + 32 * tp + 8 * g4 + 4 * hh);
          const f32x4 y = act4s<VAR>((f32x4){hc[tp][4 * g4], hc[tp][4 * g4 + 1], hc[tp][4 * g4 + 2],
                                             hc[tp][4 * g4 + 3]}, c2, K2, ik2, act);
#pragma unroll
          for (int u = 0; u < 4; ++u) part += w2[u] * y[u];
        }
    } else {
      f32x16 hc[NT];
      acc_from_bias<NT>(hc, sm.bias + 2 * H, hh);
      chain_prec_fill<PREC, NT, ENFLOW_FPM2, XD>(W, L.wc1f, L.wc1x, L.wc1b, e, hc, lane, [&](int step) {
        const int t = step >> 2, g4 = step & 3;
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = c * e[t][4 * g4 + u];
        if constexpr (MSG_LDS) {
          float* const sp = scr + j * MSP + 32 * (t & 1) + 8 * g4 + 4 * hh;
#pragma unroll
          for (int u = 0; u < 4; ++u) sp[u] = v[u];
        } else {
          f32x4* const slot = reinterpret_cast<f32x4*>(rowp + 32 * t + 8 * g4);
          const f32x4 old = *slot;
          seg_scan4(v[0], v[1], v[2], v[3], SM);
          if (seg_end) *slot = old + (f32x4){v[0], v[1], v[2], v[3]};
        }
        if (t + 1 < NT && !v_att) {
          const f32x4 y = act4s<VAR>((f32x4){e[t + 1][4 * g4], e[t + 1][4 * g4 + 1], e[t + 1][4 * g4 + 2],
                                             e[t + 1][4 * g4 + 3]}, c1, K1, ik1, act);
#pragma unroll
          for (int u = 0; u < 4; ++u) e[t + 1][4 * g4 + u] = y[u];
        }
      }, [&] { reduce_chunk(0); }, [&](int, const f16x8& bh, const f16x8&) {
        if constexpr (GUARD) o2 = or_hi(o2, bh);
      });
      reduce_chunk(NT == 4 ? 1 : 0);
      seen_big(o2, BIGK_M);
      // coord_nn.2 as a per-pair dot
#pragma unroll
      for (int tp = 0; tp < NT; ++tp)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 w2 = *reinterpret_cast<const f32x4*>(sm.bias + 3 * H + 32 * tp + 8 * g4 + 4 * hh);
          const f32x4 y = act4s<VAR>((f32x4){hc[tp][4 * g4], hc[tp][4 * g4 + 1], hc[tp][4 * g4 + 2],
                                             hc[tp][4 * g4 + 3]}, c2, K2, ik2, act);
#pragma unroll
          for (int u = 0; u < 4; ++u) part += w2[u] * y[u];
        }
    }
    float phi = part + __shfl_xor(part, 32, 64);
    if constexpr (PREC != PREC_F32) range_bad |= valid && !__builtin_isfinite(phi);
    if (v_tanh) phi = tanhf(phi);                        // egcl.py:40-42
    // norm_diff: coord_diff / (|coord_diff| + 1) (egcl.py:82-84; radial stays unnormalised)
    const float nd = v_nd ? __builtin_amdgcn_rcpf(sqrtf(radial) + 1.f) : 1.f;
    // trans = clamp(coord_diff * phi, -100, 100) (egcl.py:71-72); segment sums
    // for the mean (egcl.py:73-74); lane half 0 stores
    f32x4* const fslot = reinterpret_cast<f32x4*>(dst_row + H);   // H + 3 is padding (tw = 0)
    const f32x4 fold = *fslot;
    float tx = c * clamp100(dx * nd * phi);
    float ty = c * clamp100(dy * nd * phi);
    float tz = c * clamp100(dz * nd * phi);
    float tw = 0.f;
    seg_scan4x(tx, ty, tz, tw, SE);
    if (seg_end && hh == 0) *fslot = fold + (f32x4){tx, ty, tz, tw};
    STAMP(14);
  }
  if constexpr (PREC != PREC_F32) {
    if (__ballot(range_bad))
      if (lane == 0) atomicOr(&sm.err, ENFLOW_ERR_RANGE);
  }
  if constexpr (GUARD) {
    if (lane == 0 && t1 > t0) atomicOr(&sm.big, bigw | (uint32_t)BIGK_EDGE);
  }
  pre();
  __syncthreads();
  STAMP(15);
  // ordered fix-up of rows that continue across a wave boundary
  for (int f = tid; f < H + 3; f += BLOCK) {
    for (int ww = 0; ww < WAVES; ++ww)
      if (sm.ishead[ww]) sm.agg[sm.headrow[ww] * AST + f] += sm.head[ww][f];
  }
  __syncthreads();
}

// Q and G of the block's atoms from the per-wave partials (fixed order)
template <int H, int NMAX, int RB>
__device__ __forceinline__ void node_partials_reduce(Smem<H, NMAX, RB>& sm, const float* __restrict__ Lp,
                                                     const EgclLayout& L, int nf, int tid, int r0, int rb) {
  constexpr int NT = H / 32;
  const float bv2 = Lp[L.bv2];
  for (int a = tid; a < rb; a += BLOCK) {
    float s = 0.f;
#pragma unroll
    for (int tp = 0; tp < NT; ++tp) s += sm.u.nd.qp[tp][a];
    sm.Q[r0 + a] = s + bv2;
  }
  for (int e = tid; e < rb * nf; e += BLOCK) {
    const int a = e / nf, q = e - a * nf;
    float s = 0.f;
#pragma unroll
    for (int tp = 0; tp < NT; ++tp) s += sm.u.nd.gp[tp][q][a];
    sm.G[(r0 + a) * NFP + q] = s + Lp[L.bn2 + q];
  }
  __syncthreads();
}

// Node part of EGCL (egcl.py:26-30, 51-54, 62-67, 90-92), all on MFMA with
// atoms on the pair lanes: wave item (tp, atom tile) computes
//   Q partial   = vel_scaling_nn.2[32tp..] . silu(vel_scaling_nn.0 h)   (32 features)
//   act         = silu(node_nn.0 [h, agg])                               (32 features)
//   G partial   = node_nn.2[:, 32tp..] . act
// and the NT partials are summed in fixed order (deterministic).
template <int H, int NMAX, int RB, bool VAR = false>
__device__ __forceinline__ void node_phase(Smem<H, NMAX, RB>& sm, const float* __restrict__ Lp, const EgclLayout& L,
                                           int n, int nf, int tid, int r0, int rb) {
  constexpr int NT = H / 32;
  constexpr int NA = RB / 32;
  constexpr int AST = Smem<H, NMAX, RB>::AST;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave index: SGPR
  const int j = lane & 31, hh = lane >> 5;
  const int nh = (nf + 1) >> 1;
  const rsrc_t W = weights_rsrc(Lp, L.total);
  const Act act = VAR ? act_of(Lp + L.vfl + 1) : act_silu();
  for (int item = w; item < NT * NA; item += WAVES) {
    const int tp = item % NT, at = item / NT;
    const int a = at * 32 + j;              // row within the block
    const bool va = a < rb;
    const int ac = va ? a : 0;
    const int ag = r0 + ac;                 // atom
    // vel_scaling_nn: Q partial over this wave's 32 hidden features
    f32x16 acc = (f32x16)0.f;
    for (int s = 0; s < nh; ++s) {
      const float b = va ? sm.h[ag * NFP + 2 * s + hh] : 0.f;
      acc = mfma32(bload(W, lane * 4, (L.wv1f + (tp * (NFMAX / 2) + s) * 64) * 4), b, acc);
    }
    float part = 0.f;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int f0 = 32 * tp + 8 * g4 + 4 * hh;
      const f32x4 b1 = bload4(W, (f0 - 32 * tp) * 4, (L.bv1 + 32 * tp) * 4);   // lane part in voffset
      const f32x4 w2 = bload4(W, (f0 - 32 * tp) * 4, (L.wv2 + 32 * tp) * 4);
#pragma unroll
      for (int u = 0; u < 4; ++u) part += w2[u] * act_v<VAR>(act, acc[4 * g4 + u] + b1[u]);
    }
    part += __shfl_xor(part, 32, 64);
    if (hh == 0 && va) sm.u.nd.qp[tp][a] = part;
    // node_nn.0 over [h, agg]
    acc = (f32x16)0.f;
    for (int s = 0; s < nh; ++s) {
      const float b = va ? sm.h[ag * NFP + 2 * s + hh] : 0.f;
      acc = mfma32(bload(W, lane * 4, (L.wn1h + (tp * (NFMAX / 2) + s) * 64) * 4), b, acc);
    }
    const float* arow = &sm.agg[ac * AST];
#pragma unroll
    for (int sg = 0; sg < H / 8; ++sg) {
      const f32x4 a4 = bload4(W, lane * 16, (L.wn1a + (tp * (H / 8) + sg) * 256) * 4);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float b = va ? arow[2 * (4 * sg + u) + hh] : 0.f;
        acc = mfma32(a4[u], b, acc);
      }
    }
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 b1 = bload4(W, (8 * g4 + 4 * hh) * 4, (L.bn1 + 32 * tp) * 4);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[4 * g4 + u] = act_v<VAR>(act, acc[4 * g4 + u] + b1[u]);
    }
    // node_nn.2 partial: rows q = rho(r, hh), only r < NFMAX / 2 (q < NFMAX) can be < nf
    f32x16 gacc = (f32x16)0.f;
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const f32x4 a4 = bload4(W, lane * 16, (L.wn2f + (tp * 4 + rg) * 256) * 4);
#pragma unroll
      for (int u = 0; u < 4; ++u) gacc = mfma32(a4[u], acc[4 * rg + u], gacc);
    }
    if (va) {
#pragma unroll
      for (int r = 0; r < NFMAX / 2; ++r) {
        const int q = rho(r, hh);
        if (q < nf) sm.u.nd.gp[tp][q][a] = gacc[r];
      }
    }
  }
  __syncthreads();
  node_partials_reduce(sm, Lp, L, nf, tid, r0, rb);
}

// F16X3 node phase: same items and outputs as node_phase, all products on
// v_mfma_f32_32x32x16_f16 with hi/lo split operands (atoms on the pair lanes).
// node_phase_x3's weight fragments of one item (vel_scaling_nn.0, node_nn.0 h / agg
// parts, node_nn.2): requested up front, one L2 round trip per item
template <int H>
struct NodeFrags {
  static constexpr int NT = H / 32, KS = H / 16;
  f32x4 vh, vl, nh, nl, gfh[2], gfl[2], ah[KS], al[KS];
  __device__ __forceinline__ void issue(rsrc_t W, const EgclLayout& L, int lane, int item) {
    const int tp = item % NT, vo = lane * 32;
    vh = bload4(W, vo, (L.wv1x + tp * 512) * 4);
    vl = bload4(W, vo + 16, (L.wv1x + tp * 512) * 4);
    nh = bload4(W, vo, (L.wn1hx + tp * 512) * 4);
    nl = bload4(W, vo + 16, (L.wn1hx + tp * 512) * 4);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      gfh[s2] = bload4(W, vo, (L.wn2x + (tp * 2 + s2) * 512) * 4);
      gfl[s2] = bload4(W, vo + 16, (L.wn2x + (tp * 2 + s2) * 512) * 4);
    }
#pragma unroll
    for (int d = 0; d < KS; ++d) {
      ah[d] = bload4(W, vo, (L.wn1ax + (tp * KS + d) * 512) * 4);
      al[d] = bload4(W, vo + 16, (L.wn1ax + (tp * KS + d) * 512) * 4);
    }
  }
};

template <int H, int NMAX, int RB, bool VAR = false>
__device__ __forceinline__ void node_phase_x3_f(Smem<H, NMAX, RB>& sm, const float* __restrict__ Lp,
                                                const EgclLayout& L, int n, int nf, int tid, int r0, int rb,
                                                NodeFrags<H>& F, bool issued);
// issued: the caller requested this wave's first item (F.issue(.., wave)) before
// the edge tiles' closing barrier, so its L2 round trip overlaps the wait there
template <int H, int NMAX, int RB, bool VAR = false>
__device__ __forceinline__ void node_phase_x3(Smem<H, NMAX, RB>& sm, const float* __restrict__ Lp, const EgclLayout& L,
                                              int n, int nf, int tid, int r0, int rb) {
  NodeFrags<H> F;
  node_phase_x3_f<H, NMAX, RB, VAR>(sm, Lp, L, n, nf, tid, r0, rb, F, false);
}
template <int H, int NMAX, int RB, bool VAR>
__device__ __forceinline__ void node_phase_x3_f(Smem<H, NMAX, RB>& sm, const float* __restrict__ Lp,
                                                const EgclLayout& L, int n, int nf, int tid, int r0, int rb,
                                                NodeFrags<H>& F, bool issued) {
  constexpr int NT = H / 32;
  constexpr int NA = RB / 32;
  constexpr int AST = Smem<H, NMAX, RB>::AST;
  constexpr int KS = H / 16;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave index: SGPR
  const int j = lane & 31, hh = lane >> 5;
  const rsrc_t W = weights_rsrc(Lp, L.total);
  const float inv_v1 = Lp[L.scl + 7], inv_n1 = Lp[L.scl + 9], inv_n2 = Lp[L.scl + 11];
  const Act act = VAR ? act_of(Lp + L.vfl + 1) : act_silu();
  // every fragment of the wave's first item is requested before the bias
  // staging barrier (or earlier, by the caller), so the L2 round trips overlap
  // instead of serialising
  f32x4 &vh = F.vh, &vl = F.vl, &nh = F.nh, &nl = F.nl;
  auto& gfh = F.gfh;
  auto& gfl = F.gfl;
  auto& ah = F.ah;
  auto& al = F.al;
  auto issue = [&](int it) { F.issue(W, L, lane, it); };
  if (!issued && w < NT * NA) issue(w);
  uint32_t bigw = 0u;   // small-operand guard (BIGK_*), wave-uniform
  // vel_scaling_nn.0 / .2 and node_nn.0 biases staged in LDS (edge_tiles' bias
  // image is free now)
  for (int k = tid; k < H; k += BLOCK) {
    sm.bias[k] = Lp[L.bv1 + k];
    sm.bias[H + k] = Lp[L.wv2 + k];
    sm.bias[2 * H + k] = Lp[L.bn1 + k];
  }
  __syncthreads();
  for (int item = w; item < NT * NA; item += WAVES) {
    const int tp = item % NT, at = item / NT;
    const int a = at * 32 + j;              // row within the block
    const bool va = a < rb;
    const int ac = va ? a : 0;
    const int ag = r0 + ac;                 // atom
    // h operand (k = feature 8 hh + jj: lane half 1 holds features 8..15, zero for nf <= 8)
    f32x16 hin;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) hin[jj] = (va && 8 * hh + jj < nf) ? sm.h[ag * NFP + 8 * hh + jj] : 0.f;
    f16x8 hh16, hl16;
    split_f16(hin, 0, hh16, hl16);
    const uint32_t oh = or_hi(0u, hh16);
    uint32_t oa = oh, on = 0u;
    // vel_scaling_nn: Q partial over this wave's 32 hidden features
    f32x16 acc = (f32x16)0.f;
    acc = mfma_f16(vh, hh16, acc);
    acc = mfma_f16(vh, hl16, acc);
    acc = mfma_f16(vl, hh16, acc);
    float part = 0.f;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int f0 = 32 * tp + 8 * g4 + 4 * hh;
      const f32x4 b1 = ld4(sm.bias + f0);
      const f32x4 w2 = ld4(sm.bias + H + f0);
#pragma unroll
      for (int u = 0; u < 4; ++u) part += w2[u] * act_v<VAR>(act, fmaf(acc[4 * g4 + u], inv_v1, b1[u]));
    }
    part += __shfl_xor(part, 32, 64);
    if (hh == 0 && va) sm.u.nd.qp[tp][a] = part;
    // node_nn.0 over [h, agg]
    acc = (f32x16)0.f;
    acc = mfma_f16(nh, hh16, acc);
    acc = mfma_f16(nh, hl16, acc);
    acc = mfma_f16(nl, hh16, acc);
    const float* arow = &sm.agg[ac * AST];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      f32x16 av;
      {   // two ds_read_b128 (rows 16-B aligned, AST % 4 == 0); invalid atoms read row 0, zeroed
        static_assert(AST % 4 == 0, "node phase reads agg rows as float4");
        const f32x4 a0 = ld4(arow + 16 * ks + 8 * hh), a1 = ld4(arow + 16 * ks + 8 * hh + 4);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          av[jj] = va ? a0[jj] : 0.f;
          av[4 + jj] = va ? a1[jj] : 0.f;
        }
      }
      f16x8 bh, bl;
      split_f16(av, 0, bh, bl);
      oa = or_hi(oa, bh);
      acc = mfma_f16(ah[ks], bh, acc);
      acc = mfma_f16(ah[ks], bl, acc);
      acc = mfma_f16(al[ks], bh, acc);
    }
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 b1 = ld4(sm.bias + 2 * H + 32 * tp + 8 * g4 + 4 * hh);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[4 * g4 + u] = act_v<VAR>(act, fmaf(acc[4 * g4 + u], inv_n1, b1[u]));
    }
    // node_nn.2 partial: rows q = rho(r, hh), only r < NFMAX / 2 (q < NFMAX) can be < nf
    f32x16 gacc = (f32x16)0.f;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      f16x8 bh, bl;
      split_f16(acc, s2, bh, bl);
      on = or_hi(on, bh);
      gacc = mfma_f16(gfh[s2], bh, gacc);
      gacc = mfma_f16(gfh[s2], bl, gacc);
      gacc = mfma_f16(gfl[s2], bh, gacc);
    }
    {   // padding atoms do not count
      const uint32_t vm = va ? ENFLOW_BIG_BITS : 0u;
      bigw |= (__ballot((oh & vm) != 0u) ? (uint32_t)BIGK_HV : 0u) |
              (__ballot((oa & vm) != 0u) ? (uint32_t)BIGK_HA : 0u) |
              (__ballot((on & vm) != 0u) ? (uint32_t)BIGK_NH : 0u);
    }
    if (item + WAVES < NT * NA) issue(item + WAVES);
    if (va) {
#pragma unroll
      for (int r = 0; r < NFMAX / 2; ++r) {
        const int q = rho(r, hh);
        if (q < nf) sm.u.nd.gp[tp][q][a] = gacc[r] * inv_n2;
      }
    }
  }
  if (lane == 0 && w < NT * NA) atomicOr(&sm.big, bigw | (uint32_t)BIGK_NODE);
  __syncthreads();
  node_partials_reduce(sm, Lp, L, nf, tid, r0, rb);
}

// dequant_kernel's LDS image (round 6): only what argmax_dequant touches -- the
// molecule's h rows, network.2.weight, the activation rows of a chunk of RB
// atoms, the chunk's network outputs -- ~29 KB at H = 128 (the flow image is
// ~65 KB): five workgroups per CU, the bench batch's 1024 molecules in one
// round instead of two.  network.2.weight is staged in LDS exactly when the
// fused image stages it (<= 32 atoms): the output sums then run in the fused
// form's order, so both forms give bitwise the same z
template <int H, int NMAX, int RB>
struct DqSmem {
  static constexpr int HIDDEN_AU = 4;   // atoms per LDS round trip in the hidden layer
  static constexpr int AST = H + 4;
  static constexpr bool W1X_LDS = NMAX <= 32;
  float h[NMAX * NFP];
  alignas(16) float w1x[W1X_LDS ? 2 * NFMAX * (H + 4) : 4];
  alignas(16) float agg[RB * AST];
  struct { float net[RB * 2 * NFMAX]; } u;
  float red[WAVES];
};

// The dequantiser's draws made in the kernel (noise == NULL): Philox4x32-10
// (Salmon et al., SC'11) keyed by the caller's 64-bit seed, counter = (element
// index, 0, 64-bit offset); N(0,1) by Box-Muller (argmax.py:16's torch.randn),
// U[0,1) for Floor (floor.py's torch.rand).  Element index = atom * nf + q.
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
  }
  return c;
}
struct NoiseSrc {
  const float* buf;              // caller's draws, or NULL: drawn here
  unsigned long long seed, offset;
  __device__ __forceinline__ uint4 bits(size_t e) const {
    return philox4x32_10(make_uint4((uint32_t)e, (uint32_t)(e >> 32), (uint32_t)offset, (uint32_t)(offset >> 32)),
                         (uint32_t)seed, (uint32_t)(seed >> 32));
  }
  __device__ __forceinline__ float normal(size_t e) const {
    if (buf) return buf[e];
    const uint4 r = bits(e);
    const float u1 = (float)((r.x >> 8) + 1u) * 5.9604644775390625e-8f;   // (0, 1]
    const float u2 = (float)(r.y >> 8) * 5.9604644775390625e-8f;          // [0, 1)
    return sqrtf(-2.f * logf(u1)) * cosf(6.2831853071795865f * u2);
  }
  __device__ __forceinline__ float uniform(size_t e) const {
    if (buf) return buf[e];
    return (float)(bits(e).x >> 8) * 5.9604644775390625e-8f;
  }
};

// ArgMax.forward (enflow/nn/argmax.py:13-25) on the molecule in LDS.  h <- z;
// returns this thread's share of log_q (without the -0.5 log(2 pi) batch term).
// PAR: the last step one (atom, feature) element per thread (the split instance:
// eight waves, one molecule); else one atom per thread, its elements in turn
// (the whole-tile instances: the parallel form measured no faster there and
// moved register spills into the layer loop, profiles/r05/r05w_*, r05z2 PMC)
// S: the flow kernels' Smem image, or DqSmem (dequant_kernel's own image)
// atoms per step of argmax_dequant's hidden layer: S::HIDDEN_AU where the image
// names it (dequant_kernel: four, its rows read before any activation is
// stored), else one (inside the fused kernels the blocked form measured ~1 %
// slower on the split instance, profiles/r06/r06o_*)
template <class S, class = void>
struct HiddenAU { static constexpr int v = 1; };
template <class S>
struct HiddenAU<S, std::void_t<decltype(S::HIDDEN_AU)>> { static constexpr int v = S::HIDDEN_AU; };
// dqst (diagnostic stamps builds, dequant_kernel only): per-phase cycles, [7] the last stamp
#ifdef ENFLOW_STAMPS
#define DQS(k)                                              \
  do {                                                      \
    if (dqst) {                                             \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
      dqst[k] += now_ - dqst[7];                            \
      dqst[7] = now_;                                       \
    }                                                       \
  } while (0)
#else
#define DQS(k) do {} while (0)
#endif
template <int H, int NMAX, int RB, bool VAR = false, bool PAR = false, class S>
__device__ __forceinline__ float argmax_dequant(S& sm, const float* __restrict__ Dp, const NoiseSrc noise,
                                int a0, int n, int nf, unsigned long long* dqst = nullptr) {
#ifdef ENFLOW_ABLATE_DEQUANT
  return 0.f;   // timing ablation (tools, never the product: build.py refuses it): h passes through
#endif
  constexpr int NG = BLOCK / H > 0 ? BLOCK / H : 1;
  // hidden activations staged in agg (free before layer 0); 16-B aligned rows
  constexpr int ACT = S::AST % 4 == 0 ? S::AST : H + 1;
  static_assert(S::AST >= ACT && ACT >= H, "agg too small for the ArgMax activations");
  float* const act = sm.agg;
  const AmLayout L = argmax_layout(H, nf);
  const int tid = threadIdx.x;
  float* net = sm.u.net;
  constexpr int NETA_U = RB;                     // atoms per chunk
  float lq = 0.f;
  const Act aact = VAR ? act_of(Dp + L.act) : act_silu();   // network.1 (argmax.py:7)
  // network.2.weight staged in the (still unused) edge_nn.0 fragment buffer: the
  // output loop then reads both operands as float4 from LDS.  Rows padded to
  // WST = H + 4 floats: the output rows o a wave reads at once then start 4
  // banks apart (stride H put all of them on one bank group: a 10-way conflict
  // per ds_read_b128, ~8 k cycles of the dequantisation, profiles/r06/r06l_dq_stamps)
  constexpr int WST = H + 4;
  constexpr bool WLDS = S::W1X_LDS && ACT % 4 == 0 && sizeof(sm.w1x) >= sizeof(float) * 2 * NFMAX * WST;
  if constexpr (WLDS) {
    for (int e = tid; e < 2 * nf * H / 4; e += BLOCK) {
      const int o = 4 * e / H, k = 4 * e - o * H;
      st4(&sm.w1x[o * WST + k], ld4(Dp + L.wa2 + 4 * e));
    }
  }
  DQS(0);
  for (int c0 = 0; c0 < n; c0 += RB) {   // atoms in chunks of RB (the agg image)
    const int cn = min(RB, n - c0);
    {
      const int k = tid % H, grp = tid / H;
      if (grp < NG) {
        // network.0's column k in registers, requested once: inside the atom loop
        // the loads (a runtime-length inner loop) were issued per atom, each
        // iteration waiting on an L2 round trip (~9 k cycles of a ~30 k-cycle
        // dequantisation, profiles/r06/r06l_dq_stamps.txt); the same fma sequence (q ascending)
        const float b = Dp[L.ba1 + k];
        float w1[NFMAX];
#pragma unroll
        for (int q = 0; q < NFMAX; ++q) w1[q] = q < nf ? Dp[L.wa1t + q * H + k] : 0.f;
        // AU atoms per step, their h rows read before any activation is stored
        // (one LDS round trip per AU atoms; the same fma sequence per atom)
        constexpr int AU = HiddenAU<S>::v;
        for (int a = grp; a < cn; a += AU * NG) {
          float v[AU];
#pragma unroll
          for (int j = 0; j < AU; ++j) {
            const int aj = min(a + j * NG, cn - 1);
            v[j] = b;
#pragma unroll
            for (int q = 0; q < NFMAX; ++q)
              if (q < nf) v[j] += w1[q] * sm.h[(c0 + aj) * NFP + q];
          }
#pragma unroll
          for (int j = 0; j < AU; ++j)
            if (a + j * NG < cn) act[(a + j * NG) * ACT + k] = act_v<VAR>(aact, v[j]);
        }
      }
    }
    DQS(1);
    __syncthreads();
    DQS(2);
    // net[a][o], o < 2 nf
    for (int e = tid; e < cn * 2 * nf; e += BLOCK) {
      const int a = e / (2 * nf), o = e - a * 2 * nf;
      float s = Dp[L.ba2 + o];
      if constexpr (WLDS) {
        f32x4 acc4 = (f32x4)0.f;
#pragma unroll 8
        for (int k = 0; k < H; k += 4) {
          const f32x4 w4 = ld4(&sm.w1x[o * WST + k]), x4 = ld4(&act[a * ACT + k]);
          acc4 += w4 * x4;
        }
        s += (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
      } else {
        const float* wr = Dp + L.wa2 + o * H;
        for (int k = 0; k < H; ++k) s += wr[k] * act[a * ACT + k];
      }
      net[a * 2 * NFMAX + o] = s;          // chunk-local rows
    }
    DQS(3);
    __syncthreads();
    DQS(2);
    if constexpr (!PAR) {
      for (int a = tid; a < cn; a += BLOCK) {   // z of the chunk's atoms (each atom's own h only)
        const int ag = c0 + a;
        float u[NFMAX], hv[NFMAX];
        float T = 0.f;
#pragma unroll
        for (int q = 0; q < NFMAX; ++q) {
          if (q < nf) {
            const float ls = net[a * 2 * NFMAX + q], tr = net[a * 2 * NFMAX + nf + q];
            u[q] = tr + noise.normal((size_t)(a0 + ag) * nf + q) * expf(ls);
            hv[q] = sm.h[ag * NFP + q];
            T += hv[q] * u[q];
            lq += -0.5f * u[q] * u[q] - ls;
          }
        }
#pragma unroll
        for (int q = 0; q < NFMAX; ++q) {
          if (q < nf) {
            const float z = hv[q] * u[q] + (1.f - hv[q]) * (T - softplus_f(T - u[q]));
            lq -= (1.f - hv[q]) * logsigmoid_f(T - u[q]);
            sm.h[ag * NFP + q] = z;
          }
        }
      }
      __syncthreads();
    } else {
      // z of the chunk's atoms (each atom's own h only), one (atom, feature)
      // element per thread: the draw (Philox + Box-Muller) and exp of every element
      // in parallel rather than an atom's nf elements in turn on one thread; u
      // staged in the (consumed) activation rows, T = sum_q h_q u_q in feature order
      // by each element's thread, z staged before h is overwritten
      static_assert(S::AST * RB >= 2 * NETA_U * NFMAX, "u / z staging fits the activation rows");
      float* const us = act;                       // [a][q] u
      float* const zs = act + NETA_U * NFMAX;      // [a][q] z
      for (int e = tid; e < cn * nf; e += BLOCK) {
        const int a = e / nf, q = e - a * nf, ag = c0 + a;
        const float ls = net[a * 2 * NFMAX + q], tr = net[a * 2 * NFMAX + nf + q];
        const float u = tr + noise.normal((size_t)(a0 + ag) * nf + q) * expf(ls);
        us[a * NFMAX + q] = u;
        lq += -0.5f * u * u - ls;
      }
      DQS(4);
      __syncthreads();
      DQS(2);
      for (int e = tid; e < cn * nf; e += BLOCK) {
        const int a = e / nf, q = e - a * nf, ag = c0 + a;
        float T = 0.f;
        for (int q2 = 0; q2 < nf; ++q2) T += sm.h[ag * NFP + q2] * us[a * NFMAX + q2];
        const float hv = sm.h[ag * NFP + q], u = us[a * NFMAX + q];
        zs[a * NFMAX + q] = hv * u + (1.f - hv) * (T - softplus_f(T - u));
        lq -= (1.f - hv) * logsigmoid_f(T - u);
      }
      DQS(5);
      __syncthreads();
      for (int e = tid; e < cn * nf; e += BLOCK) {
        const int a = e / nf, q = e - a * nf;
        sm.h[(c0 + a) * NFP + q] = zs[a * NFMAX + q];
      }
      __syncthreads();
      DQS(6);
    }
  }
  return lq;
}

// deterministic block sum (thread values -> one float, fixed order)
template <class S>
__device__ __forceinline__ float block_sum(S& sm, float v) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sm.red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int k = 0; k < WAVES; ++k) s += sm.red[k];
  return s;
}

struct FlowArgs {
  const int32_t* mol_ptr;
  const float* r_cut;
  const float* box;
  float* h;
  float* g;
  float* pos;
  float* vel;
  const float* layers;
  int n_layers;
  int nf;
  int dequant_kind;
  const float* dequant;
  const float* noise;
  float dequant_scale;
  float dt;
  float cw;
  float* ldj_mol;
  int32_t* argmax_idx;
  int32_t* max_idx;
  int32_t* err;
  unsigned long long* stats;   // optional: [0] += unique pairs, [1] += reference edges
  float* tape;                 // optional (training): TapeLayout block
  int32_t* pair_counts;        // optional (training): [n_layers][num_mols] unique pairs
  int num_mols, num_atoms;
  // ABI 8 (out-of-place, self-contained forward): inputs read from *_in when set
  // (the outputs h / g / pos / vel are then written only); noise == NULL draws
  // in the kernel (NoiseSrc); ticket != NULL: the last workgroup to finish
  // reduces ldj_mol into ldj_total (+ ldj_cst) and resets the ticket
  const float* h_in = nullptr;
  const float* g_in = nullptr;
  const float* pos_in = nullptr;
  const float* vel_in = nullptr;
  unsigned long long seed = 0, offset = 0;
  uint32_t* ticket = nullptr;
  float* ldj_total = nullptr;
  double ldj_cst = 0.0;
  // ABI 12: per-molecule error words (OR of the molecule's ENFLOW_ERR_* bits; the
  // caller zeroes them), and a molecule list (block b runs molecule mol_list[b])
  int32_t* mol_err = nullptr;
  const int32_t* mol_list = nullptr;
  // round 6: the ArgMax dequantisation ran ahead of the flow kernel
  // (dequant_kernel): the flow gets dequant_kind NONE, h_in = z, and adds each
  // molecule's log_q from here to its log|detJ|
  const float* lq_mol = nullptr;
  __device__ __forceinline__ NoiseSrc noise_src() const { return NoiseSrc{noise, seed, offset}; }
};

enum { LOAD_POS = 1, LOAD_H = 2, LOAD_VELG = 4 };

template <int H, int NMAX, int RB>
__device__ __forceinline__ bool load_molecule(Smem<H, NMAX, RB>& sm, const FlowArgs& A, MolRef& M, int what) {
  const int m = A.mol_list ? A.mol_list[blockIdx.x] : (int)blockIdx.x;
  const int tid = threadIdx.x;
  M.m = m;
  M.a0 = A.mol_ptr[m];
  M.n = A.mol_ptr[m + 1] - M.a0;
  M.rc = 0.f;
  M.bx = M.by = M.bz = 0.f;
  if (M.n > NMAX || A.nf > NFMAX) {
    if (tid == 0) {
      const int e = M.n > NMAX ? ENFLOW_ERR_TOO_MANY_ATOMS : ENFLOW_ERR_TOO_MANY_FEATURES;
      atomicOr(A.err, e);
      if (A.mol_err) atomicOr(&A.mol_err[m], e);
    }
    return false;
  }
  const int n = M.n, nf = A.nf;
  if (what & LOAD_POS) {
    M.rc = A.r_cut[m];
    for (int e = tid; e < n * 3; e += BLOCK) {
      sm.pos[e] = (A.pos_in ? A.pos_in : A.pos)[(size_t)M.a0 * 3 + e];
      // blocked images keep only the first atom's box (the edge box); the
      // per-atom pbc boxes are read from global memory in the update
      if (!Smem<H, NMAX, RB>::BLOCKED || e < 3) sm.boxa[e] = A.box[(size_t)M.a0 * 3 + e];
    }
  }
  if (what & LOAD_VELG)
    for (int e = tid; e < n * 3; e += BLOCK) sm.vel[e] = (A.vel_in ? A.vel_in : A.vel)[(size_t)M.a0 * 3 + e];
  const float* const hin = A.h_in ? A.h_in : A.h;
  const float* const gin = A.g_in ? A.g_in : A.g;
  for (int e = tid; e < n * NFP; e += BLOCK) {   // rows zero-padded past nf
    const int a = e / NFP, q = e - a * NFP;
    const size_t src = (size_t)(M.a0 + a) * nf + q;
    if (what & LOAD_H) sm.h[e] = q < nf ? hin[src] : 0.f;
    if (what & LOAD_VELG) sm.g[e] = q < nf ? gin[src] : 0.f;
  }
  if (tid == 0) {
    sm.err = 0;
    sm.big = 0u;
  }
  __syncthreads();
  if ((what & LOAD_POS) && n > 0) {
    M.bx = sm.boxa[0];
    M.by = sm.boxa[1];
    M.bz = sm.boxa[2];
  }
  return true;
}

