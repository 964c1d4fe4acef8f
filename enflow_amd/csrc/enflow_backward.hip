// enflow_backward.hip -- training backward of the fused coupling flow on MI355X.
//
// Reverse-mode gradient of  loss = Alchemical_NLL(LFIntegrator(data))
// (enflow/flow/loss.py:21-24, enflow/flow/dynamics.py:10-24, enflow/nn/egcl.py,
// enflow/nn/argmax.py) with respect to every parameter, i.e. what the
// reference's `loss.backward()` (enflow/main.py:219-221) produces by autograd.
//
// Data flow (one stream, no host synchronisation):
//   forward (enflow_flow.hip) with a tape: per layer the layer-input state
//     (h, g, pos, vel), the message sums and Q, plus per-molecule pair counts;
//   nll_bwd_kernel: adjoints of the flow outputs and of log|detJ|;
//   pair_offsets_kernel: 32-aligned per-molecule row offsets of every layer;
//   per layer, last to first:
//     lf_layer_bwd_kernel (one workgroup per molecule, state in LDS):
//       leapfrog adjoint -> node MLP backward (VALU, atoms x hidden units)
//       -> per 32-pair tile the edge chain is recomputed and back-propagated
//       on v_mfma_f32_32x32x2_f32 (transposed weight fragments, accumulator
//       tiles chained as B operands exactly as in the forward), writing the
//       per-pair (input, output-gradient) rows every weight gradient needs;
//     outer_acc_kernel + reduce_part_kernel: every weight gradient of the
//       layer as dW = sum_rows DY^T X (chunked over rows, fixed-order reduce,
//       deterministic), written straight into the torch parameter layout;
//   argmax_bwd_kernel (+ its two weight gradients).
// All arithmetic is float32.

#define ENFLOW_BACKWARD_TU   // -DENFLOW_STAMPS_BWD stamps this file's kernels only (tools/stamps_bwd.py)
#include "enflow_large.h"
#include <stdlib.h>

// ---------------------------------------------------------------------------
// packing of the backward weight section
// ---------------------------------------------------------------------------
__device__ __forceinline__ void pack_egcl_bwd_body(const float* __restrict__ raw, int H, int nf, float* __restrict__ out) {
  const EgclBwdLayout L = egcl_bwd_layout(H);
  const RawEgcl R = raw_egcl(H, nf);
  const int NT = H / 32;
  const int K1 = 2 * nf + 1;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < L.total; idx += gridDim.x * blockDim.x) {
    float v = 0.f;
    if (idx < L.we1T) {                     // W^T chain fragments: A[row][col] = W[col][row]
      const bool c1 = idx >= L.wc1T;
      const int e = idx - (c1 ? L.wc1T : L.we2T);
      const int u = e & 3, lane = (e >> 2) & 63, rg = (e >> 8) & 3, rest = e >> 10;
      const int t = rest % NT, tp = rest / NT;
      const int row = 32 * tp + (lane & 31), col = 32 * t + rho(4 * rg + u, lane >> 5);
      v = raw[(c1 ? R.Wc1 : R.We2) + col * H + row];
    } else if (idx < L.wv1T) {              // we1T[tp][rg][lane][4]: A[q][k] = We1[k][q]
      const int e = idx - L.we1T;
      const int u = e & 3, lane = (e >> 2) & 63, rg = (e >> 8) & 3, tp = e >> 10;
      const int q = lane & 31, k = 32 * tp + rho(4 * rg + u, lane >> 5);
      if (q < K1) v = raw[R.We1 + k * K1 + q];
    } else if (idx >= L.scl && idx < L.scl + 16) {
      continue;                             // written by egcl_bwd_scale_kernel
    } else if (idx >= L.we2Tx && idx < L.we1Tx) {   // F16X3 W^T chain fragments [tp][t][s][lane][hi|lo]
      const bool c1 = idx >= L.wc1Tx;
      const int e = idx - (c1 ? L.wc1Tx : L.we2Tx);
      const int d = e & 7, lane = (e >> 3) & 63, rest = e >> 9;
      const int sstep = rest & 1, t = (rest >> 1) % NT, tp = (rest >> 1) / NT;
      const float sc = out[L.scl + (c1 ? 2 : 0)];
      const int row = 32 * tp + (lane & 31);
      const int j0 = 2 * (d & 3);
      const int col0 = 32 * t + rho(8 * sstep + j0, lane >> 5), col1 = 32 * t + rho(8 * sstep + j0 + 1, lane >> 5);
      const int Wo = c1 ? R.Wc1 : R.We2;
      v = __builtin_bit_cast(float, f16_split_bits(raw[Wo + col0 * H + row] * sc, raw[Wo + col1 * H + row] * sc, d >= 4));
    } else if (idx >= L.we1Tx && idx < L.we1Tx + NT * 2 * 512) {   // F16X3 edge_nn.0^T [tp][s][lane][hi|lo]
      const int e = idx - L.we1Tx;
      const int d = e & 7, lane = (e >> 3) & 63, blk = e >> 9;
      const int tp = blk >> 1, s2 = blk & 1;
      const float sc = out[L.scl + 4];
      const int q = lane & 31, j0 = 2 * (d & 3);
      const int k0 = 32 * tp + rho(8 * s2 + j0, lane >> 5), k1 = 32 * tp + rho(8 * s2 + j0 + 1, lane >> 5);
      const float w0 = q < K1 ? raw[R.We1 + k0 * K1 + q] * sc : 0.f;
      const float w1 = q < K1 ? raw[R.We1 + k1 * K1 + q] * sc : 0.f;
      v = __builtin_bit_cast(float, f16_split_bits(w0, w1, d >= 4));
    } else if (idx >= L.wn2Tx && idx < L.wn1aTx + NT * (H / 16) * 512) {   // F16X3 node-backward fragments
      int e, sidx;
      if (idx < L.wvTx) { e = idx - L.wn2Tx; sidx = 0; }
      else if (idx < L.wnhTx) { e = idx - L.wvTx; sidx = 1; }
      else if (idx < L.wn1aTx) { e = idx - L.wnhTx; sidx = 2; }
      else { e = idx - L.wn1aTx; sidx = 3; }
      const int d = e & 7, lane = (e >> 3) & 63, blk = e >> 9;
      const int m = lane & 31, kh = lane >> 5;
      const float sc = out[L.scl + (sidx == 0 ? 10 : (sidx == 1 ? 6 : 8))];
      float w2[2];
      for (int q = 0; q < 2; ++q) {
        const int jj = 2 * (d & 3) + q;
        float w = 0.f;
        if (sidx == 0) {                 // blk = tp; k index = aG feature
          const int f = 8 * kh + jj;
          if (f < nf) w = raw[R.Wn2 + f * H + 32 * blk + m];
        } else if (sidx < 3) {           // blk = tp * 2 + s; rows f < nf
          const int tp = blk >> 1, s2 = blk & 1;
          const int k = 32 * tp + rho(8 * s2 + jj, kh);
          if (m < nf) w = sidx == 1 ? raw[R.Wv1 + k * nf + m] : raw[R.Wn1 + k * (H + nf) + m];
        } else {                         // blk = tp * (H / 16) + ks
          const int tp = blk / (H / 16), ks = blk % (H / 16);
          const int k = 16 * ks + 8 * kh + jj;
          w = raw[R.Wn1 + k * (H + nf) + nf + 32 * tp + m];
        }
        w2[q] = w * sc;
      }
      v = __builtin_bit_cast(float, f16_split_bits(w2[0], w2[1], d >= 4));
    } else if (idx < L.wn1T) {              // wv1T[f][k]
      const int e = idx - L.wv1T, f = e / H, k = e % H;
      if (f < nf) v = raw[R.Wv1 + k * nf + f];
    } else if (idx < L.scl) {               // wn1T[f][k]
      const int e = idx - L.wn1T, f = e / H, k = e % H;
      if (f < NFMAX) {
        if (f < nf) v = raw[R.Wn1 + k * (H + nf) + f];
      } else if (f - NFMAX < H) {
        v = raw[R.Wn1 + k * (H + nf) + nf + (f - NFMAX)];
      }
    }
    out[idx] = v;
  }
}

__global__ void pack_egcl_bwd_kernel(const float* __restrict__ raw, int H, int nf, float* __restrict__ out) {
  pack_egcl_bwd_body(raw, H, nf, out);
}
// every layer at once: layer blockIdx.y at raw + y raw_stride, out + y stride
__global__ void pack_egcl_bwd_layers_kernel(const float* __restrict__ raw, int64_t raw_stride, int H, int nf,
                                            float* __restrict__ out, int64_t stride) {
  pack_egcl_bwd_body(raw + blockIdx.y * raw_stride, H, nf, out + blockIdx.y * stride);
}

__global__ void __launch_bounds__(256) egcl_bwd_scale_kernel(const float* __restrict__ raw, int H, int nf,
                                                             float* __restrict__ out) {
  egcl_scales_block(raw, H, nf, out + egcl_bwd_layout(H).scl);
}
__global__ void __launch_bounds__(256) egcl_bwd_scale_layers_kernel(const float* __restrict__ raw, int64_t raw_stride,
                                                                    int H, int nf, float* __restrict__ out,
                                                                    int64_t stride) {
  egcl_scales_block(raw + blockIdx.y * raw_stride, H, nf, out + blockIdx.y * stride + egcl_bwd_layout(H).scl);
}

__device__ __forceinline__ float sigmoid_f(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float dsilu_f(float z) {   // d silu / dz
  const float s = sigmoid_f(z);
  return s * (1.f + z * (1.f - s));
}
// act'(z): the SiLU form above unless a generic (GEN) instance runs another act_fn
template <bool GEN>
__device__ __forceinline__ float dact_v(const Act& A, float z) {
  if (!GEN || A.k == ACT_SILU) return dsilu_f(z);
  return act_d(A, z);
}

// ---------------------------------------------------------------------------
// per-layer backward
// ---------------------------------------------------------------------------
struct BwdArgs {
  const int32_t* mol_ptr;
  const float* r_cut;
  const float* box;
  const float* tape;
  int num_atoms, num_mols, n_layers, layer, nf;
  const float* Lp;   // packed forward layer
  const float* Bp;   // packed backward section
  const float* Rp;   // raw (torch-layout) layer parameters
  float dt, cw;
  const float* adj_ldj;
  float* ah;         // [A][nf]  adjoints of h / g / pos / vel: layer output in, layer input out
  float* ag;
  float* apos;       // [A][3]
  float* avel;
  const int32_t* pair_off;   // this layer's [num_mols + 1] row offsets (32-aligned)
  // pair rows, tile-blocked (trow).  pre(edge_nn.0) and pre(coord_nn.0) are not
  // stored: this kernel recomputes pre0 for silu', outer_x3_kernel recomputes
  // pre0 from xin (X of edge_nn.2) and pre(coord_nn.0) from the message (DY of
  // coord_nn.0, X of coord_nn.2), bitwise as here.  pe is stored as the
  // pre-activation: outer_x3_kernel applies silu on load, this kernel re-reads it.
  float* xin;        // [P][16] h_i, h_j, radial                     (X of edge_nn.0)
  float* p0;         // unused (ABI <= 7 layout)
  float* pe;         // [P][H] pre(edge_nn.2)           silu -> X of coord_nn.0 (the message)
  float* pc;         // unused
  float* dp0;        // [P][H] d pre(edge_nn.0)                      (DY of edge_nn.0)
  float* dpe;        // [P][H] d pre(edge_nn.2)                      (DY of edge_nn.2)
  float* aphi;       // [P]    d phi                                 (DY of coord_nn.2)
  float* patt;       // [P]    att of the pair (VAR; 1 without attention): X of coord_nn.0 is e * att
  float* dlogit;     // [P]    d att_nn logit (VAR; 0 without attention) (DY of att_nn.0)
  float* tmax;       // [P / 32][TMX_W] per 32-row tile: max |operand| of the pair-row weight-gradient
                     // products (TMX_*), the scales outer_x3_kernel puts on a whole chunk
  float* su;         // atom rows [A][H] silu(vel_scaling_nn.0)      (X of vel_scaling_nn.2)
  float* au;         // [A][H] d pre(vel_scaling_nn.0)               (DY of vel_scaling_nn.0)
  float* sn;         // [A][H] silu(node_nn.0)                       (X of node_nn.2)
  float* an;         // [A][H] d pre(node_nn.0)                      (DY of node_nn.0)
  float* aq;         // [A]    dQ                                    (DY of vel_scaling_nn.2)
  float* agr;        // [A][nf] dG                                   (DY of node_nn.2)
  int32_t* err;
  // standalone EGCL.forward backward (enflow_egcl_backward_f32): adjoints of the
  // network outputs Q [A], F [A][3], G [A][nf] given directly (NULL: the flow's
  // leapfrog adjoint); the layer-input adjoints then start at zero
  // fused path: the forward taped the layer's pair words / row counts (TapeLayout::pairs,
  // cnt) and its pair counts ([num_mols], this layer's): loaded, not rebuilt (0: rebuild,
  // the standalone EGCL backward's tape)
  const int32_t* pair_counts_l;
  int tape_pairs;
  const float* eg_dQ;
  const float* eg_dF;
  const float* eg_dG;
  // large systems (lf_layer_bwd_kernel<.., BIG = true>): one workgroup per block of
  // rbl rows; the rows' pair words come from the large path's neighbour search
  // (enflow_large.h), column atoms are read from the tape; each pair's column-side
  // d h / d pos goes to colc (summed per column by lg_colsum / lg_colfinal)
  const int32_t* blk_start;
  int rbl, max_n;
  const int32_t* npairs_g;    // [A] pair words of row a
  const int32_t* cntrow_g;    // [A] edges of row a
  const uint32_t* pairs_g;    // [A][max_n] (label << 5 | mult << 27)
  const int32_t* boff;        // [blocks] first pair row of the block (32-aligned)
  int32_t* rowstart;          // [A] out: first pair row of row atom a
  float* colc;                // [pair rows][CSTR] out
  long long prb;              // pair rows allocated
};
// weight-fragment ring depth of the layer backward's F16X3 chains (prefetch distance
// + 1 k-steps; each slot is 8 VGPRs of hi / lo fragments).  Depth 3 / 4 / 6 measured
// within 1 % of 2 (profiles/r04/r04l_ab_train_split_once_and_ring_depth.txt)
#ifndef ENFLOW_BWD_X3_DEPTH
#define ENFLOW_BWD_X3_DEPTH 2
#endif
#ifndef ENFLOW_BWD_RL
#define ENFLOW_BWD_RL 2   // when GEMM3 re-reads the parked pre_e rows (A/B knob, see the tile; r04u: 2 -0.8 %)
#endif
// per-tile operand maxima (BwdArgs::tmax): X / DY of edge_nn.0, edge_nn.2, coord_nn.0
enum { TMX_XIN = 0, TMX_DP0 = 1, TMX_X1 = 2, TMX_DPE = 3, TMX_MSG = 4, TMX_DPC = 5, TMX_W = 8 };
// edge_nn.0 input rows [h_i, h_j, radial]: 2 nf + 1 columns rounded up to 16
__host__ __device__ inline int xin_width(int nf) { return (2 * nf + 1 + 15) & ~15; }
constexpr int CSTR = NFMAX + 4;   // colc row: d h_j [NFMAX], d pos_j [3], pad
// the transposed edge_nn.0 GEMM (d [h_i, h_j, radial]) has one 32-row output
// tile: training needs 2 nf + 1 <= 32
// node_nf the backward takes: every feature of the build (nf 16: the radial
// row of the transposed edge_nn.0 GEMM, q = 2 nf = 32, lies past its 32-row
// output tile and is a separate dot product, see lf_layer_bwd_kernel GEMM5)
constexpr int BWD_NFMAX = NFMAX;

// <= 80 KB at (H, NMAX) = (128, 64): two workgroups per CU.  The node-MLP
// adjoint rows go through LDS a chunk of Smem::NBCH atoms at a time, in the
// union the pair build uses later.
template <int H, int NMAX>
struct BwdSmem {
  using Img = Smem<H, NMAX, NMAX, true>;
  Img f;
  float ah[NMAX * NFP], ag[NMAX * NFP], aG[NMAX * NFP];
  float apos[NMAX * 3], avel[NMAX * 3], aF[NMAX * 3];
  float aQ[NMAX];
  uint32_t nmax[NMAX / 32];   // per atom tile: max |d pre(node_nn.0)| (float bits)
  alignas(16) float wrad[NFMAX == 16 ? H : 1];   // nf 16: edge_nn.0.weight[:, 2 nf] (the radial column)
};

// Adjoint tiles span many decades (coord_nn.2 starts at gain 0.001), so before
// an F16X3 product their values are scaled by a power of two that puts the
// tile's max |x| in [2^12, 2^13): hi / lo parts stay normal fp16.  Returns the
// exact inverse scale.
template <int NT>
__device__ __forceinline__ float lane_absmax(const f32x16 (&X)[NT]) {
  float m = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) m = fmaxf(m, fabsf(X[t][r]));
  return m;
}
// m: the wave's max |x| over X (wave-uniform)
template <int NT>
__device__ __forceinline__ float tile_pow2_scale(f32x16 (&X)[NT], float m) {
  int ex = 0;
  if (m > 0.f && isfinite(m)) {
    frexpf(m, &ex);
    ex = 13 - ex;
    ex = ex > 100 ? 100 : (ex < -100 ? -100 : ex);
  }
  const float s = ldexpf(1.f, ex);
#pragma unroll
  for (int t = 0; t < NT; ++t) X[t] *= s;
  return ldexpf(1.f, -ex);
}
template <int NT>
__device__ __forceinline__ float tile_pow2_scale(f32x16 (&X)[NT]) {
  return tile_pow2_scale(X, wave_max(lane_absmax(X)));
}


// power of two putting m in [2^12, 2^13) (0 for m == 0 / non-finite)
__device__ __forceinline__ int pow2_exp(float m) {
  int ex = 0;
  if (m > 0.f && isfinite(m)) {
    frexpf(m, &ex);
    ex = 13 - ex;
    ex = ex > 100 ? 100 : (ex < -100 ? -100 : ex);
  }
  return ex;
}

// Node MLPs backward on F16X3 MFMA, atoms on the lanes (the forward's node
// phase transposed): per item (32 hidden units tp, 32 atoms at) the
// pre-activations of vel_scaling_nn.0 and node_nn.0 are recomputed, d pre of
// both (rows su / au / sn / an for the weight gradients), then
//   d h   += vel_scaling_nn.0.weight^T d u + node_nn.0.weight[:, :nf]^T d pre
//            (per-item partials, fixed-order sum over tp),
//   d agg  = node_nn.0.weight[:, nf:]^T d pre   (into sm.agg, over the message sums).
// Adjoint operands carry power-of-two scales like the edge chain's.
template <int H, int NMAX, bool VAR = false>
__device__ __forceinline__ void node_bwd_x3(BwdSmem<H, NMAX>& sb, const BwdArgs& B, const EgclLayout& L,
                                            const EgclBwdLayout& LB, int a0, int n, int nf, int tid) {
  auto& sm = sb.f;
  constexpr int NT = H / 32, NA = NMAX / 32, KS = H / 16, NI = NT * NA, IPW = (NI + WAVES - 1) / WAVES;
  constexpr int AST = BwdSmem<H, NMAX>::Img::AST;
  static_assert(NT * NFMAX * NMAX <= BwdSmem<H, NMAX>::Img::NBW, "dh partials do not fit sm.u.nb");
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hh = lane >> 5;
  const rsrc_t W = weights_rsrc(B.Lp, L.total), WB = weights_rsrc(B.Bp, LB.total);
  const int vo = lane * 32;
  const float inv_v1 = B.Lp[L.scl + 7], inv_n1 = B.Lp[L.scl + 9], inv_n2 = B.Lp[L.scl + 11];
  const Act act = VAR ? act_of(B.Lp + L.vfl + 1) : act_silu();
  float* const gp = sm.u.nb;   // d h partials [tp][q][atom]
  for (int k = tid; k < H; k += BLOCK) {
    sm.bias[k] = B.Lp[L.bv1 + k];
    sm.bias[H + k] = B.Lp[L.wv2 + k];
    sm.bias[2 * H + k] = B.Lp[L.bn1 + k];
  }
  if (tid < NA) sb.nmax[tid] = 0u;
  __syncthreads();
  auto mm3 = [&](const rsrc_t& r, int off_floats, const f16x8& bh, const f16x8& bl, f32x16 acc) {
    const f32x4 ah = bload4(r, vo, off_floats * 4), al = bload4(r, vo + 16, off_floats * 4);
    acc = mfma_f16(ah, bh, acc);
    acc = mfma_f16(ah, bl, acc);
    return mfma_f16(al, bh, acc);
  };
  f32x16 keep[IPW];
#pragma unroll
  for (int ii = 0; ii < IPW; ++ii) {
    const int item = w + WAVES * ii;
    if (item >= NI) break;
    const int tp = item % NT, at = item / NT;
    const int a = at * 32 + j;
    const bool va = a < n;
    const int ac = va ? a : 0;
    f32x16 hin = (f32x16)0.f, gin = (f32x16)0.f;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {   // k = feature 8 hh + jj (half 1: features 8..15)
      const bool on = va && 8 * hh + jj < nf;
      hin[jj] = on ? sm.h[ac * NFP + 8 * hh + jj] : 0.f;
      gin[jj] = on ? sb.aG[ac * NFP + 8 * hh + jj] : 0.f;
    }
    f16x8 bh, bl;
    split_f16(hin, 0, bh, bl);
    f32x16 zu = mm3(W, L.wv1x + tp * 512, bh, bl, (f32x16)0.f);
    f32x16 zn = mm3(W, L.wn1hx + tp * 512, bh, bl, (f32x16)0.f);
    const float* arow = &sm.agg[ac * AST];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      f32x16 av;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) av[jj] = va ? arow[16 * ks + 8 * hh + jj] : 0.f;
      split_f16(av, 0, bh, bl);
      zn = mm3(W, L.wn1ax + (tp * KS + ks) * 512, bh, bl, zn);
    }
    // d silu(node_nn.0) = node_nn.2.weight^T d G
    f32x16 gs[1] = {gin};
    const float ig = tile_pow2_scale(gs);
    split_f16(gs[0], 0, bh, bl);
    const f32x16 asn = mm3(WB, LB.wn2Tx + tp * 512, bh, bl, (f32x16)0.f);
    const float ug = inv_n2 * ig;
    const float aq = va ? sb.aQ[ac] : 0.f;
    f32x16 au, an;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int f0 = 32 * tp + 8 * g4 + 4 * hh;
      const f32x4 b1 = ld4(sm.bias + f0), w2 = ld4(sm.bias + H + f0), bn = ld4(sm.bias + 2 * H + f0);
      f32x4 su4, au4, sn4, an4;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = 4 * g4 + u;
        const float z1 = fmaf(zu[r], inv_v1, b1[u]), z2 = fmaf(zn[r], inv_n1, bn[u]);
        float f1, f2, d1, d2;
        act_fd<VAR>(act, z1, f1, d1);
        act_fd<VAR>(act, z2, f2, d2);
        su4[u] = f1;
        sn4[u] = f2;
        au4[u] = aq * w2[u] * d1;
        an4[u] = asn[r] * ug * d2;
        au[r] = au4[u];
        an[r] = an4[u];
      }
      if (va) {
        const size_t row = (size_t)(a0 + a) * H + f0;
        st4(B.su + row, su4);
        st4(B.au + row, au4);
        st4(B.sn + row, sn4);
        st4(B.an + row, an4);
      }
    }
    // d h partial over this item's hidden units (rows f = rho(r, hh) < nf: r < NFMAX / 2)
    f32x16 tu[1] = {au}, tn[1] = {an};
    const float iu = tile_pow2_scale(tu), in = tile_pow2_scale(tn);
    f32x16 dv = (f32x16)0.f, dn = (f32x16)0.f;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      split_f16(tu[0], s2, bh, bl);
      dv = mm3(WB, LB.wvTx + (tp * 2 + s2) * 512, bh, bl, dv);
      split_f16(tn[0], s2, bh, bl);
      dn = mm3(WB, LB.wnhTx + (tp * 2 + s2) * 512, bh, bl, dn);
    }
    if (va) {
#pragma unroll
      for (int r = 0; r < NFMAX / 2; ++r) {
        const int q = rho(r, hh);
        if (q < nf) gp[(tp * NFMAX + q) * NMAX + a] = dv[r] * (inv_v1 * iu) + dn[r] * (inv_n1 * in);
      }
    }
    keep[ii] = an;
    float mx = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, fabsf(an[r]));
    mx = wave_max(mx);
    if (lane == 0) atomicMax(&sb.nmax[at], __float_as_uint(mx));
  }
  __syncthreads();   // message-sum rows consumed; partials and tile maxima complete
  // d pre(node_nn.0) rows into sm.agg, scaled per atom tile
#pragma unroll
  for (int ii = 0; ii < IPW; ++ii) {
    const int item = w + WAVES * ii;
    if (item >= NI) break;
    const int tp = item % NT, at = item / NT, a = at * 32 + j;
    const float s = ldexpf(1.f, pow2_exp(__uint_as_float(sb.nmax[at])));
    if (a < n) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sm.agg[a * AST + 32 * tp + rho(r, hh)] = keep[ii][r] * s;
    }
  }
  for (int e = tid; e < n * nf; e += BLOCK) {   // d h: fixed-order sum over the hidden tiles
    const int a = e / nf, q = e - a * nf;
    float acc = 0.f;
#pragma unroll
    for (int tp = 0; tp < NT; ++tp) acc += gp[(tp * NFMAX + q) * NMAX + a];
    sb.ah[a * NFP + q] += acc;
  }
  __syncthreads();
  // d agg = node_nn.0.weight[:, nf:]^T d pre
#pragma unroll
  for (int ii = 0; ii < IPW; ++ii) {
    const int item = w + WAVES * ii;
    if (item >= NI) break;
    const int tp = item % NT, at = item / NT, a = at * 32 + j;
    const bool va = a < n;
    const float* arow = &sm.agg[(va ? a : 0) * AST];
    f32x16 acc = (f32x16)0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      f32x16 av;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) av[jj] = va ? arow[16 * ks + 8 * hh + jj] : 0.f;
      f16x8 bh, bl;
      split_f16(av, 0, bh, bl);
      acc = mm3(WB, LB.wn1aTx + (tp * KS + ks) * 512, bh, bl, acc);
    }
    keep[ii] = acc * (inv_n1 * ldexpf(1.f, -pow2_exp(__uint_as_float(sb.nmax[at]))));
  }
  __syncthreads();   // d pre rows consumed
#pragma unroll
  for (int ii = 0; ii < IPW; ++ii) {
    const int item = w + WAVES * ii;
    if (item >= NI) break;
    const int tp = item % NT, at = item / NT, a = at * 32 + j;
    if (a < n) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sm.agg[a * AST + 32 * tp + rho(r, hh)] = keep[ii][r];
    }
  }
  __syncthreads();
}

#ifndef ENFLOW_BWD_PREC
#define ENFLOW_BWD_PREC PREC_F16X3
#endif
// timing ablations (tools/ab_train.py; results are wrong): 1 = drop the pair-row
// output stores, 2 = also drop the parked silu' rows
#ifndef ENFLOW_BWD_ABLATE
#define ENFLOW_BWD_ABLATE 0
#endif
#define ST_OUT(r, vo, so, v) do { if (!(ENFLOW_BWD_ABLATE & 1)) bstore(r, vo, so, v); } while (0)
#define ST_PARK(r, vo, so, v) do { if (!(ENFLOW_BWD_ABLATE & 2)) bstore(r, vo, so, v); } while (0)

// Pair rows are stored tile-blocked: the 32 rows of a tile are contiguous per
// feature, element (row p, feature f) of a W-wide array at
// ((p / 32) * W + f) * 32 + p % 32.  A wave's accumulator register (one
// feature per half-wave, pairs on the lanes) is then two full 128-byte lines,
// and outer_acc_kernel reads a tile as one contiguous W x 32 block.
__device__ __forceinline__ size_t trow(size_t rtile, int W, int f, int j) {
  return ((rtile * W + f) << 5) + j;
}
// VAR: layers may carry EGCL_NORM_DIFF / EGCL_TANH (read per layer from the
// packed forward layer; a second instance so the default kernel keeps its
// register allocation).  EGCL_ATTENTION is refused by the host.
template <int H, int NMAX, bool VAR = false, int PREC = ENFLOW_BWD_PREC, bool BIG = false>
__global__ void __launch_bounds__(BLOCK, 2) lf_layer_bwd_kernel(BwdArgs B) {
  static_assert(PREC == PREC_F32 || PREC == PREC_F16X3, "backward: fp32-accurate precisions only");
  static_assert(!BIG || NMAX == 32, "large systems: 32-row blocks");
  __shared__ BwdSmem<H, NMAX> sb;
  __shared__ int roff[BIG ? 33 : 1];   // BIG: the rows' first pair word within the block
  using Img = typename BwdSmem<H, NMAX>::Img;
  Img& sm = sb.f;
  constexpr int NT = H / 32;
  constexpr int AST = Img::AST;
  constexpr int NBCH = Img::NBCH;
  const int tid = threadIdx.x;
  // fused: m = the molecule, a0 / n its atoms.  BIG: a0 / n = the block's rows,
  // ma0 / mn = their molecule's atoms
  int m, a0, n, ma0, mn;
  if constexpr (BIG) {
    const int b = blockIdx.x;
    if (b >= B.blk_start[B.num_mols]) return;
    m = seg_of(B.blk_start, B.num_mols, b);
    ma0 = B.mol_ptr[m];
    mn = B.mol_ptr[m + 1] - ma0;
    const int r0 = (b - B.blk_start[m]) * B.rbl;
    a0 = ma0 + r0;
    n = min(B.rbl, mn - r0);
  } else {
    m = blockIdx.x;
    a0 = B.mol_ptr[m];
    n = B.mol_ptr[m + 1] - a0;
    ma0 = a0;
    mn = n;
  }
  if (n > NMAX || B.nf > BWD_NFMAX) {
    if (tid == 0) atomicOr(B.err, n > NMAX ? ENFLOW_ERR_TOO_MANY_ATOMS : ENFLOW_ERR_TOO_MANY_FEATURES);
    return;
  }
  const int nf = B.nf;
  const float dt = B.dt;
  const EgclLayout L = egcl_layout(H, nf);
  const EgclBwdLayout LB = egcl_bwd_layout(H);
  const RawEgcl R = raw_egcl(H, nf);
  const TapeLayout T = tape_layout(B.num_atoms, nf, H, B.n_layers);
  const size_t la = (size_t)B.layer * B.num_atoms + a0;
  const float* Rp = B.Rp;
  const float* Bp = B.Bp;

  STAMP_DECL
  // ---- layer-input state (tape), message sums, Q; adjoints of the layer output
  for (int e = tid; e < n * 3; e += BLOCK) {
    sm.pos[e] = B.tape[T.pos + la * 3 + e];
    sm.vel[e] = B.tape[T.vel + la * 3 + e];
    sm.boxa[e] = B.box[(size_t)a0 * 3 + e];
    sb.apos[e] = B.apos[(size_t)a0 * 3 + e];
    sb.avel[e] = B.avel[(size_t)a0 * 3 + e];
  }
  for (int e = tid; e < n * NFP; e += BLOCK) {
    const int a = e / NFP, q = e - a * NFP;
    const bool v = q < nf;
    sm.h[e] = v ? B.tape[T.hx + (la + a) * T.ldhx + q] : 0.f;
    sm.g[e] = v ? B.tape[T.g + (la + a) * nf + q] : 0.f;
    sb.ah[e] = v ? B.ah[(size_t)(a0 + a) * nf + q] : 0.f;
    sb.ag[e] = v ? B.ag[(size_t)(a0 + a) * nf + q] : 0.f;
  }
  for (int e = tid; e < n * H; e += BLOCK) {
    const int a = e / H, k = e - a * H;
    sm.agg[a * AST + k] = B.tape[T.hx + (la + a) * T.ldhx + nf + k];
  }
  for (int a = tid; a < n; a += BLOCK) sm.Q[a] = B.tape[T.q + la + a];
  if (tid == 0) sm.err = 0;
  if constexpr (BIG) {
    for (int a = tid; a < n; a += BLOCK) sm.cntrow[a] = B.cntrow_g[a0 + a];
    if (tid == 0) {
      int acc = 0;
      for (int a = 0; a < n; ++a) { roff[a] = acc; acc += B.npairs_g[a0 + a]; }
      for (int a = n; a <= 32; ++a) roff[a] = acc;
    }
  }
  __syncthreads();
  if constexpr (BIG) {   // the host's pair-row bound comes from the forward's counts
    if ((long long)B.boff[blockIdx.x] + ((roff[32] + 31) & ~31) > B.prb) {
      if (tid == 0) atomicOr(B.err, ENFLOW_ERR_TOO_MANY_ATOMS);
      return;
    }
    for (int a = tid; a < n; a += BLOCK) B.rowstart[a0 + a] = B.boff[blockIdx.x] + roff[a];
  }
  MolRef M;
  M.a0 = ma0;
  M.n = mn;
  M.rc = B.r_cut[m];
  if constexpr (BIG) {   // the molecule's edge box: its first atom's (base.py:130)
    M.bx = B.box[(size_t)ma0 * 3 + 0];
    M.by = B.box[(size_t)ma0 * 3 + 1];
    M.bz = B.box[(size_t)ma0 * 3 + 2];
  } else {
    M.bx = n > 0 ? sm.boxa[0] : 0.f;
    M.by = n > 0 ? sm.boxa[1] : 0.f;
    M.bz = n > 0 ? sm.boxa[2] : 0.f;
  }

  STAMP(0);
  // ---- leapfrog adjoint (dynamics.py:13-21 in reverse order)
  const float aldj = B.adj_ldj[0];
  if (B.eg_dQ) {   // EGCL.forward alone (egcl.py:76-92): d Q / d F / d G given
    for (int a = tid; a < n; a += BLOCK) {
      sb.aQ[a] = B.eg_dQ[a0 + a];
      for (int d = 0; d < 3; ++d) {
        sb.aF[a * 3 + d] = B.eg_dF[(size_t)(a0 + a) * 3 + d];
        sb.apos[a * 3 + d] = 0.f;
        sb.avel[a * 3 + d] = 0.f;
      }
      for (int q = 0; q < NFP; ++q) {
        sb.aG[a * NFP + q] = q < nf ? B.eg_dG[(size_t)(a0 + a) * nf + q] : 0.f;
        sb.ah[a * NFP + q] = 0.f;
        sb.ag[a * NFP + q] = 0.f;
      }
    }
  } else
  for (int a = tid; a < n; a += BLOCK) {
    const float eq = expf(sm.Q[a]);
    float s = 0.f;
    for (int d = 0; d < 3; ++d) {
      const float avt = sb.avel[a * 3 + d] + sb.apos[a * 3 + d] * dt;   // pos' = pbc(pos + vel' dt)
      s += sm.vel[a * 3 + d] * avt;
      sb.avel[a * 3 + d] = eq * avt;                                   // vel' = e^Q vel + F dt
      sb.aF[a * 3 + d] = avt * dt;
    }
    sb.aQ[a] = eq * s + aldj;                                          // + ldj += Q.sum()
    for (int q = 0; q < nf; ++q) {
      const float agt = sb.ag[a * NFP + q] + sb.ah[a * NFP + q] * dt;  // h' = h + g' dt
      sb.ag[a * NFP + q] = agt;                                        // g' = g + G dt
      sb.aG[a * NFP + q] = agt * dt;
    }
  }
  __syncthreads();

  STAMP(1);
  // ---- node MLPs backward (egcl.py:26-30, 51-54, 90-92)
  for (int a = tid; a < n; a += BLOCK) B.aq[a0 + a] = sb.aQ[a];
  for (int e = tid; e < n * nf; e += BLOCK) {
    const int a = e / nf, q = e - a * nf;
    B.agr[(size_t)a0 * nf + e] = sb.aG[a * NFP + q];
  }
  if constexpr (PREC == PREC_F16X3) {
    node_bwd_x3<H, NMAX, VAR>(sb, B, L, LB, a0, n, nf, tid);
  } else {
  // VALU form (fp32 mode), NBCH atoms at a time:
  //      threads = (hidden unit k, atom group); adjoint rows staged in sm.u.nb
  {
    constexpr int NG = BLOCK / H;
    const int k = tid % H, grp = tid / H;
    const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const float bv1 = Rp[R.bv1 + k], bn1 = Rp[R.bn1 + k], wv2 = Rp[R.Wv2 + k];
    for (int c0 = 0; c0 < n; c0 += NBCH) {
      const int c1 = min(n, c0 + NBCH);
      for (int a = c0 + grp; a < c1; a += NG) {
        float u = bv1, nn = bn1;
        for (int f = 0; f < nf; ++f) {
          const float hv = sm.h[a * NFP + f];
          u = fmaf(Bp[LB.wv1T + f * H + k], hv, u);
          nn = fmaf(Bp[LB.wn1T + f * H + k], hv, nn);
        }
        const float* arow = &sm.agg[a * AST];
        const float* wcol = Bp + LB.wn1T + NFMAX * H + k;
#pragma unroll 8
        for (int f = 0; f < H; ++f) nn = fmaf(wcol[f * H], arow[f], nn);
        const Act act = VAR ? act_of(B.Lp + L.vfl + 1) : act_silu();
        float su_v, sn_v, du, dn;
        act_fd<VAR>(act, u, su_v, du);
        act_fd<VAR>(act, nn, sn_v, dn);
        const float au = sb.aQ[a] * wv2 * du;
        float asn = 0.f;
        for (int q = 0; q < nf; ++q) asn = fmaf(Rp[R.Wn2 + q * H + k], sb.aG[a * NFP + q], asn);
        const float an = asn * dn;
        const size_t row = (size_t)(a0 + a) * H + k;
        B.su[row] = su_v;
        B.au[row] = au;
        B.sn[row] = sn_v;
        B.an[row] = an;
        sm.u.nb[(a - c0) * 2 * H + k] = au;
        sm.u.nb[(a - c0) * 2 * H + H + k] = an;
      }
      __syncthreads();
      // d agg = node_nn.0.weight[:, nf:]^T d pre  (overwrites the chunk's message sums)
      for (int a = c0 + grp; a < c1; a += NG) {
        const float* anr = &sm.u.nb[(a - c0) * 2 * H + H];
        const float* wr = Rp + R.Wn1 + nf + k;
        float s = 0.f;
#pragma unroll 8
        for (int kk = 0; kk < H; ++kk) s = fmaf(wr[kk * (H + nf)], anr[kk], s);
        sm.agg[a * AST + k] = s;
      }
      // d h += vel_scaling_nn.0.weight^T d u + node_nn.0.weight[:, :nf]^T d pre:
      // one (atom, feature) per wave step, hidden units over the lanes
      for (int e = w; e < (c1 - c0) * nf; e += WAVES) {
        const int al = e / nf, f = e - al * nf;
        const float* aur = &sm.u.nb[al * 2 * H];
        float s = 0.f;
        for (int kk = lane; kk < H; kk += 64)
          s += Rp[R.Wv1 + kk * nf + f] * aur[kk] + Rp[R.Wn1 + kk * (H + nf) + f] * aur[H + kk];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (lane == 0) sb.ah[(c0 + al) * NFP + f] += s;
      }
      __syncthreads();
    }
  }
  }
  STAMP(2);
  for (int k = tid; k < H; k += BLOCK) {   // edge-chain biases (the node phase used sm.bias)
    sm.bias[k] = B.Lp[L.be1 + k];
    sm.bias[H + k] = B.Lp[L.be2 + k];
    sm.bias[2 * H + k] = B.Lp[L.bc1 + k];
    sm.bias[3 * H + k] = B.Lp[L.wc2 + k];
    if constexpr (NFMAX == 16) {
      if (2 * nf + 1 > 32) sb.wrad[k] = Rp[R.We1 + k * (2 * nf + 1) + 2 * nf];
    }
  }
  if constexpr (!BIG) {
    if (B.tape_pairs) {   // the forward's list of this layer (same positions -> the same pairs)
      const int np = B.pair_counts_l[m];
      const float* tp = B.tape + T.pairs + la * TAPE_PAIR_CAP;
      for (int e = tid; e < np; e += BLOCK) sm.pairs[e] = __float_as_uint(tp[e]);
      for (int a = tid; a < n; a += BLOCK) sm.cntrow[a] = __float_as_int(B.tape[T.cnt + la + a]);
      if (tid == 0) sm.npairs = np;
      __syncthreads();
    } else {
      build_pairs(sm, M, tid);   // same positions as the forward -> same pairs (reuses sm.u)
    }
  }

  STAMP(3);
  // ---- edge chain backward, one 32-pair tile per wave step (egcl.py:57-74, 76-89)
  {
    const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave index: SGPR
    const int j = lane & 31, hh = lane >> 5;
    const int P_all = BIG ? roff[32] : sm.npairs;   // pairs of the molecule / row block
    const int TT_all = (P_all + 31) >> 5;
    const rsrc_t W = weights_rsrc(B.Lp, L.total);
    const rsrc_t WB = weights_rsrc(B.Bp, LB.total);
    const float hbx = M.bx * 0.5f, hby = M.by * 0.5f, hbz = M.bz * 0.5f;
    const size_t prow0 = BIG ? (size_t)B.boff[blockIdx.x] : (size_t)B.pair_off[m];
    // BIG: column atoms from the tape (this layer's input state of the molecule)
    const float* cpos = B.tape + T.pos + ((size_t)B.layer * B.num_atoms + ma0) * 3;
    const float* chx = B.tape + T.hx + ((size_t)B.layer * B.num_atoms + ma0) * T.ldhx;
    const bool x3 = PREC == PREC_F16X3;
    const float inv1 = x3 ? B.Lp[L.scl + 1] : 1.f;   // edge_nn.2 / coord_nn.0 / edge_nn.0 (and ^T)
    const float inv2 = x3 ? B.Lp[L.scl + 3] : 1.f;
    const float inv0 = x3 ? B.Lp[L.scl + 5] : 1.f;
    auto nofill = [](int) {};
    const int vfl = VAR ? (int)B.Lp[L.vfl] : 0;   // wave-uniform constructor variants
    const bool v_nd = VAR && (vfl & EGCL_NORM_DIFF) != 0, v_tanh = VAR && (vfl & EGCL_TANH) != 0;
    const bool v_att = VAR && (vfl & EGCL_ATTENTION) != 0;
    const Act act = VAR ? act_of(B.Lp + L.vfl + 1) : act_silu();   // act_fn (egcl.py:11)
    // the molecule's tile-blocked rows (trow): buffer resources on its first
    // row, per element a wave-uniform byte offset (tile, feature) + the lane's
    const size_t nrow = (size_t)TT_all * 32;
    const rsrc_t rpe = rows_rsrc(B.pe + prow0 * H, nrow * H);
    const rsrc_t rdp0 = rows_rsrc(B.dp0 + prow0 * H, nrow * H), rdpe = rows_rsrc(B.dpe + prow0 * H, nrow * H);
    // edge_nn.0 input rows [h_i, h_j, radial]: 16 wide, 32 when 2 nf + 1 > 16 (nf = 8)
    const int XW = xin_width(nf);
    const rsrc_t rxin = rows_rsrc(B.xin + prow0 * XW, nrow * XW);
    const int lob = (hh * 128 + j) * 4;   // lane bytes: (feature 4hh, row j)
    // d h / d pos of the edge part: each wave adds into its own [atom][nf + 3]
    // slab (one wave's LDS atomics apply in a fixed order), summed over the
    // waves in wave order afterwards -> bitwise reproducible
    const int EW = nf + 3;
    float* const wacc = sm.u.nb + (size_t)w * n * EW;
    for (int e = tid; e < WAVES * n * EW; e += BLOCK) sm.u.nb[e] = 0.f;
    __syncthreads();
    constexpr int PCAP = Img::PC;   // BIG: pair words per pass through sm.pairs
    static_assert(PCAP % 32 == 0, "passes of whole tiles");
    for (int pp0 = 0;; pp0 += PCAP) {
    int P = P_all;
    if constexpr (BIG) {   // the next pass of the rows' pair words (| local row)
      P = min(PCAP, P_all - pp0);
      for (int e = tid; e < P; e += BLOCK) {
        const int pe = pp0 + e;
        int lo = 0, hi = n;   // row il: roff[il] <= pe < roff[il + 1]
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (roff[mid] <= pe) lo = mid;
          else hi = mid;
        }
        sm.pairs[e] = B.pairs_g[(size_t)(a0 + lo) * B.max_n + (pe - roff[lo])] | (uint32_t)lo;
      }
      __syncthreads();
    }
    const int TT = (P + 31) >> 5;
    const int tpw = (TT + WAVES - 1) / WAVES;
    const int t0 = w * tpw, t1 = min(TT, t0 + tpw);
    // GEMM0's first-k-step weight fragments (the same for every tile): loaded
    // here, re-requested by each tile's second GEMM0 and carried into the next
    // tile's first, which then waits on no load
    f32x4 cfh[NT], cfl[NT];
    if constexpr (PREC == PREC_F16X3) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int so = (L.we1x + (t * KS0MAX) * 512) * 4;
        cfh[t] = bload4(W, lane * 32, so);
        cfl[t] = bload4(W, lane * 32 + 16, so);
      }
    }
    for (int tile = t0; tile < t1; ++tile) {
      const int p = tile * 32 + j;
      const bool valid = p < P;
      const uint32_t pr = valid ? sm.pairs[p] : 0u;
      int i, jl;
      float c;   // multiplicity; 0 on padding lanes
      if constexpr (BIG) {
        i = (int)(pr & 31u);
        jl = (int)((pr >> 5) & 0x3fffffu);
        c = (float)(pr >> 27);
      } else {
        i = (int)(pr & 0xffu);
        jl = (int)((pr >> 8) & 0xffu);
        c = (float)(pr >> 16);
      }
      const int gt = (pp0 >> 5) + tile;   // tile index within the molecule's / block's rows
      const size_t Rw = prow0 + (size_t)(pp0 + p);
      // the tile's max |operand| of each weight-gradient product (outer_x3_kernel's
      // chunk scales): wave-reduced, lane 0 stores
      float* const tmx = B.tmax + ((prow0 >> 5) + (size_t)gt) * TMX_W;
      auto put_max = [&](int op, float m) {
        m = wave_max(m);
        if (lane == 0) tmx[op] = m;
        return m;
      };
      const int tsb = gt * H * 128;   // tile byte offset in an H-wide array (16-wide: / (H / 16))
      float cx, cy, cz;   // column atom position
      if constexpr (BIG) {
        cx = cpos[jl * 3 + 0];
        cy = cpos[jl * 3 + 1];
        cz = cpos[jl * 3 + 2];
      } else {
        cx = sm.pos[jl * 3 + 0];
        cy = sm.pos[jl * 3 + 1];
        cz = sm.pos[jl * 3 + 2];
      }
      auto colh = [&](int q) -> float {   // column atom feature q < nf
        if constexpr (BIG) return chx[(size_t)jl * T.ldhx + q];
        else return sm.h[jl * NFP + q];
      };
      const float dx = pbc1(sm.pos[i * 3 + 0] - cx, hbx);
      const float dy = pbc1(sm.pos[i * 3 + 1] - cy, hby);
      const float dz = pbc1(sm.pos[i * 3 + 2] - cz, hbz);
      const float radial = dx * dx + dy * dy + dz * dz;

      // X row of edge_nn.0: [h_i, h_j, radial]
      float mxin = valid ? radial : 0.f;
      auto xin_col = [&](int q) -> float {
        float v = 0.f;
        if (q < nf) v = sm.h[i * NFP + q];
        else if (q < 2 * nf) v = colh(q - nf);
        else if (q == 2 * nf) v = radial;
        v = valid ? v : 0.f;
        mxin = fmaxf(mxin, fabsf(v));
        return v;
      };
      if constexpr (NFMAX == 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) ST_OUT(rxin, (hh * 256 + j) * 4, gt * XW * 128 + u * 128, xin_col(8 * hh + u));
        if (XW > 16 && hh == 0)   // q = 16 = 2 nf: the radial of an nf = 8 layer
          ST_OUT(rxin, j * 4, gt * XW * 128 + 16 * 128, valid ? radial : 0.f);
      } else {   // 16-column chunks, every column of the row written
        for (int c16 = 0; c16 < XW / 16; ++c16)
#pragma unroll
          for (int u = 0; u < 8; ++u)
            ST_OUT(rxin, (hh * 256 + j) * 4, gt * XW * 128 + (16 * c16 + u) * 128, xin_col(16 * c16 + 8 * hh + u));
      }
      put_max(TMX_XIN, mxin);

      // GEMM0 (recompute): pre0 = edge_nn.0 [h_i, h_j, radial] + be1.  Run twice per
      // tile (here, and again for silu'(pre0) after GEMM4) instead of parking pre0
      // in HBM: the same instruction sequence on the same operands, so both are
      // bitwise the forward's pre0 (outer_x3_kernel recomputes it from xin, too)
      auto gemm0 = [&](f32x16 (&x0)[NT], bool fresh) {
#pragma unroll
      for (int t = 0; t < NT; ++t) x0[t] = (f32x16)0.f;
      if constexpr (PREC == PREC_F16X3) {
        const int ks_n = gemm0_ksteps(nf), nch = gemm0_nch(nf);
        // the first k-step's fragments: carried (cfh / cfl), or requested before
        // the operand build so their L2 round trip overlaps it
        auto& fh0 = cfh;
        auto& fl0 = cfl;
        if (fresh) {
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const int so = (L.we1x + (t * KS0MAX) * 512) * 4;
            fh0[t] = bload4(W, lane * 32, so);
            fl0[t] = bload4(W, lane * 32 + 16, so);
          }
        }
        for (int ks = 0; ks < ks_n; ++ks) {   // k order gemm0_col (as the forward)
          f32x16 in;
          if (ks < nch) {
            const int f0 = 8 * ks;
            if (BIG && hh) {
#pragma unroll
              for (int jj = 0; jj < 8; ++jj) in[jj] = f0 + jj < nf ? colh(f0 + jj) : 0.f;
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
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            f32x4 ah = fh0[t], al = fl0[t];
            if (ks) {
              const int so = (L.we1x + (t * KS0MAX + ks) * 512) * 4;
              ah = bload4(W, lane * 32, so);
              al = bload4(W, lane * 32 + 16, so);
            }
            x0[t] = mfma_f16(ah, bh, x0[t]);
            x0[t] = mfma_f16(ah, bl, x0[t]);
            x0[t] = mfma_f16(al, bh, x0[t]);
          }
        }
        const float inv0 = B.Lp[L.scl + 5];
#pragma unroll
        for (int t = 0; t < NT; ++t) x0[t] *= inv0;
      } else {
#pragma unroll
        for (int s = 0; s < NFMAX + 1; ++s) {
          const int qc = 2 * (s - NFMAX / 2) + hh;
          const float b = s < NFMAX / 2 ? sm.h[i * NFP + 2 * s + hh]
                        : (s < NFMAX ? (BIG ? (qc < nf ? colh(qc) : 0.f) : sm.h[jl * NFP + qc])
                                     : (hh == 0 ? radial : 0.f));
#pragma unroll
          for (int t = 0; t < NT; ++t)
            x0[t] = mfma32(bload(W, lane * 4, (L.we1f + (t * (NFMAX + 1) + s) * 64) * 4), b, x0[t]);
        }
      }
      };
      f32x16 x0[NT];
      gemm0(x0, false);
      STAMP(4);
      // x1 = silu(pre0) (kept: B operand of GEMM1)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int f0 = 32 * t + 8 * g4 + 4 * hh;
          const f32x4 b = ld4(sm.bias + f0);
#pragma unroll
          for (int u = 0; u < 4; ++u) x0[t][4 * g4 + u] = act_v<VAR>(act, x0[t][4 * g4 + u] + b[u]);
        }
      put_max(TMX_X1, lane_absmax(x0));
      __builtin_amdgcn_sched_barrier(0);   // keep the stage's stores ahead of the next chain
      STAMP(5);
      // GEMM1 (recompute): e = silu(edge_nn.2 x1 + be2); pre_e stored
      f32x16 ev[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) ev[t] = (f32x16)0.f;
      chain_prec_fill<PREC, NT, 1, ENFLOW_BWD_X3_DEPTH>(W, L.we2f, L.we2x, L.we2b, x0, ev, lane, nofill);
      STAMP(18);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int f0 = 32 * t + 8 * g4 + 4 * hh;
          const f32x4 b = ld4(sm.bias + H + f0);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float z = fmaf(ev[t][4 * g4 + u], inv1, b[u]);
            ST_PARK(rpe, lob, tsb + ((32 * t + 8 * g4 + u) << 7), z);
            ev[t][4 * g4 + u] = act_v<VAR>(act, z);
          }
        }
      float att = 1.f;
      if (v_att) {   // egcl.py:60-62: message = e * sigmoid(att_nn(e))
        float d = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const f32x4 wa = ld4(B.Lp + L.watt + 32 * t + 8 * g4 + 4 * hh);
#pragma unroll
            for (int u = 0; u < 4; ++u) d = fmaf(wa[u], ev[t][4 * g4 + u], d);
          }
        att = sigm_f(d + __shfl_xor(d, 32, 64) + B.Lp[L.batt]);
#pragma unroll
        for (int t = 0; t < NT; ++t) ev[t] *= att;
      }
      put_max(TMX_MSG, lane_absmax(ev));
      __builtin_amdgcn_sched_barrier(0);   // keep the stage's stores ahead of the next chain
      STAMP(6);
      // GEMM2 (recompute): phi = coord_nn.2 silu(coord_nn.0 e + bc1)
      f32x16 cv[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) cv[t] = (f32x16)0.f;
      chain_prec_fill<PREC, NT, 1, ENFLOW_BWD_X3_DEPTH>(W, L.wc1f, L.wc1x, L.wc1b, ev, cv, lane, nofill);
      STAMP(19);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // pre_e rows landed
      float part = 0.f;
      float mdz = 0.f;   // max |silu'(c)| (DY of coord_nn.0 = d phi * silu'(c))
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int f0 = 32 * t + 8 * g4 + 4 * hh;
          const f32x4 b = ld4(sm.bias + 2 * H + f0);
          const f32x4 w2 = ld4(sm.bias + 3 * H + f0);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float z = fmaf(cv[t][4 * g4 + u], inv2, b[u]);
            float dz;
            if (!VAR || act.k == ACT_SILU) {
              const float s = sigmoid_f(z);
              part = fmaf(w2[u], z * s, part);   // pc is not stored: outer_x3_kernel recomputes it
              dz = s * (1.f + z * (1.f - s));    // silu'(c)
            } else {
              part = fmaf(w2[u], act_f(act, z), part);
              dz = act_d(act, z);
            }
            mdz = fmaxf(mdz, fabsf(dz));
            cv[t][4 * g4 + u] = w2[u] * dz;      // wc2 * silu'(c)
          }
        }
      float phi = part + __shfl_xor(part, 32, 64);
      if (v_tanh) phi = tanhf(phi);                             // egcl.py:40-42
      // norm_diff: trans uses coord_diff / (|coord_diff| + 1) (egcl.py:82-84)
      const float rr = v_nd ? sqrtf(radial) : 0.f;
      const float nd = v_nd ? __builtin_amdgcn_rcpf(rr + 1.f) : 1.f;
      const float dxn = dx * nd, dyn = dy * nd, dzn = dz * nd;
      // d phi from dF (egcl.py:71-74: mean over the row's edges, clamp, coords_weight)
      const float inv = B.cw / fmaxf((float)sm.cntrow[i], 1.f);
      const float gx = fabsf(dxn * phi) <= 100.f ? sb.aF[i * 3 + 0] * inv : 0.f;
      const float gy = fabsf(dyn * phi) <= 100.f ? sb.aF[i * 3 + 1] * inv : 0.f;
      const float gz = fabsf(dzn * phi) <= 100.f ? sb.aF[i * 3 + 2] * inv : 0.f;
      float aph = c * (gx * dxn + gy * dyn + gz * dzn);
      if (v_tanh) aph *= 1.f - phi * phi;                       // d of coord_nn.2's output
      if (hh == 0 && !(ENFLOW_BWD_ABLATE & 1)) B.aphi[Rw] = aph;
      if (VAR && hh == 0) B.patt[Rw] = att;
      put_max(TMX_DPC, mdz * fabsf(aph));
      // d pre(coord_nn.0) = dphi * wc2 * silu'(c)   (not stored: outer_acc rebuilds it from pc)
#pragma unroll
      for (int t = 0; t < NT; ++t) cv[t] *= aph;
      __builtin_amdgcn_sched_barrier(0);   // keep the stage's stores ahead of the next chain
      STAMP(7);
      // GEMM3: d e = c * d agg[i] + coord_nn.0.weight^T d pre(coord_nn.0)
      f32x16 ae[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) ae[t] = (f32x16)0.f;
      float sc3 = 1.f;
      if constexpr (PREC == PREC_F16X3) sc3 = tile_pow2_scale(cv);   // cv already stored unscaled
      STAMP(16);
      // pre_e rows re-read (ENFLOW_BWD_RL 0: during the chain, a quad per step;
      // 1: all before the chain; 2: all after it)
      f32x16 rl[NT];
      auto rl_load = [&](int i) {
        const int t = i >> 2, g4 = i & 3;
#pragma unroll
        for (int u = 0; u < 4; ++u) rl[t][4 * g4 + u] = bload(rpe, lob, tsb + ((32 * t + 8 * g4 + u) << 7));
      };
      if constexpr (ENFLOW_BWD_RL == 1) {
#pragma unroll
        for (int i = 0; i < 4 * NT; ++i) rl_load(i);
      }
      chain_prec_fill<PREC, NT, 1, ENFLOW_BWD_X3_DEPTH>(WB, LB.wc1T, LB.wc1Tx, 0, cv, ae, lane, [&](int i) {
        if constexpr (ENFLOW_BWD_RL == 0) rl_load(i);
      });
      if constexpr (ENFLOW_BWD_RL == 2) {
#pragma unroll
        for (int i = 0; i < 4 * NT; ++i) rl_load(i);
      }
      STAMP(17);
      const float u3 = inv2 * sc3;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) ae[t][r] = fmaf(ae[t][r], u3, c * sm.agg[i * AST + 32 * t + rho(r, hh)]);
      if constexpr (VAR) {   // ae = d message; through message = e * att
        float dl = 0.f;
        if (v_att) {
          float s = 0.f;
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) s = fmaf(ae[t][r], act_v<VAR>(act, rl[t][r]), s);   // d message . e
          dl = (s + __shfl_xor(s, 32, 64)) * att * (1.f - att);                      // d logit
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
              const f32x4 wa = ld4(B.Lp + L.watt + 32 * t + 8 * g4 + 4 * hh);
#pragma unroll
              for (int u = 0; u < 4; ++u) ae[t][4 * g4 + u] = fmaf(ae[t][4 * g4 + u], att, wa[u] * dl);
            }
        }
        if (hh == 0) B.dlogit[Rw] = dl;
      }
      STAMP(8);
      // d pre(edge_nn.2) = d e * silu'(pre_e)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int f0 = 32 * t + 8 * g4 + 4 * hh;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            ae[t][4 * g4 + u] *= dact_v<VAR>(act, rl[t][4 * g4 + u]);
            ST_OUT(rdpe, lob, tsb + ((32 * t + 8 * g4 + u) << 7), ae[t][4 * g4 + u]);
          }
        }
      __builtin_amdgcn_sched_barrier(0);   // keep the stage's stores ahead of the next chain
      STAMP(9);
      // GEMM4: d x1 = edge_nn.2.weight^T d pre(edge_nn.2);  d pre0 = d x1 * silu'(pre0)
      f32x16 ax[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) ax[t] = (f32x16)0.f;
      float sc4 = 1.f;
      const float mdpe = put_max(TMX_DPE, lane_absmax(ae));
      if constexpr (PREC == PREC_F16X3) sc4 = tile_pow2_scale(ae, mdpe);   // ae already stored unscaled
      chain_prec_fill<PREC, NT, 1, ENFLOW_BWD_X3_DEPTH>(WB, LB.we2T, LB.we2Tx, 0, ae, ax, lane, nofill);
      STAMP(10);
      gemm0(rl, true);   // pre0 again (bitwise the first pass's)
      const float u4 = inv1 * sc4;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int f0 = 32 * t + 8 * g4 + 4 * hh;
          const f32x4 b = ld4(sm.bias + f0);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            ax[t][4 * g4 + u] = ax[t][4 * g4 + u] * u4 * dact_v<VAR>(act, rl[t][4 * g4 + u] + b[u]);
            ST_OUT(rdp0, lob, tsb + ((32 * t + 8 * g4 + u) << 7), ax[t][4 * g4 + u]);
          }
        }
      __builtin_amdgcn_sched_barrier(0);   // keep the stage's stores ahead of the next chain
      STAMP(11);
      // GEMM5: d [h_i, h_j, radial] = edge_nn.0.weight^T d pre0   (rows q < 2nf+1)
      f32x16 ain = (f32x16)0.f;
      float sc5 = 1.f;
      const float mdp0 = put_max(TMX_DP0, lane_absmax(ax));
      if constexpr (PREC == PREC_F16X3) {
        sc5 = tile_pow2_scale(ax, mdp0);   // ax already stored unscaled
#pragma unroll
        for (int tp = 0; tp < NT; ++tp)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int so = (LB.we1Tx + (tp * 2 + s2) * 512) * 4;
            const f32x4 gh = bload4(WB, lane * 32, so), gl = bload4(WB, lane * 32 + 16, so);
            f16x8 bh, bl;
            split_f16(ax[tp], s2, bh, bl);
            ain = mfma_f16(gh, bh, ain);
            ain = mfma_f16(gh, bl, ain);
            ain = mfma_f16(gl, bh, ain);
          }
        ain *= inv0 * sc5;
      } else {
#pragma unroll
        for (int tp = 0; tp < NT; ++tp)
#pragma unroll
          for (int rg = 0; rg < 4; ++rg) {
            const f32x4 a4 = bload4(WB, lane * 16, (LB.we1T + (tp * 4 + rg) * 256) * 4);
#pragma unroll
            for (int u = 0; u < 4; ++u) ain = mfma32(a4[u], ax[tp][4 * rg + u], ain);
          }
      }
      STAMP(12);
      float arad = 0.f;
      // nf 16: the radial row q = 2 nf = 32 is past the 32-row tile: a dot product
      // of d pre0 (this lane half's features, scaled by 1 / sc5 in f16x3) with
      // the radial column, the two halves summed, held by lane half 0
      float arad16 = 0.f;
      if constexpr (NFMAX == 16) {
        if (2 * nf + 1 > 32) {
          float s = 0.f;
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
              const f32x4 wr = ld4(sb.wrad + 32 * t + 8 * g4 + 4 * hh);
#pragma unroll
              for (int u = 0; u < 4; ++u) s = fmaf(ax[t][4 * g4 + u], wr[u], s);
            }
          s += __shfl_xor(s, 32, 64);
          arad16 = hh == 0 ? s * sc5 : 0.f;
        }
      }
      if (valid) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int q = rho(r, hh);
          if (q < nf) atomicAdd(&wacc[i * EW + q], ain[r]);
          else if (q < 2 * nf) {
            if constexpr (BIG) B.colc[Rw * CSTR + q - nf] = ain[r];
            else atomicAdd(&wacc[jl * EW + q - nf], ain[r]);
          } else if (q == 2 * nf) arad = ain[r];
        }
        if (NFMAX == 16 && 2 * nf + 1 > 32) arad = arad16;
      }
      // d coord_diff (radial = |cd|^2, trans = cd * phi), d pos_i += ., d pos_j -= .
      const float sF = hh == 0 ? c * phi : 0.f;
      float ux = sF * gx, uy = sF * gy, uz = sF * gz;             // d (normalised) coord_diff
      if (v_nd) {   // through cd / (|cd| + 1): nd u - nd^2 (u . cd) cd / |cd|
        const float k2 = rr > 0.f ? nd * nd * (ux * dx + uy * dy + uz * dz) / rr : 0.f;
        ux = nd * ux - k2 * dx;
        uy = nd * uy - k2 * dy;
        uz = nd * uz - k2 * dz;
      }
      const float tx = ux + 2.f * dx * arad;
      const float ty = uy + 2.f * dy * arad;
      const float tz = uz + 2.f * dz * arad;
      if constexpr (BIG) {   // the column's d pos: both half-waves' parts, one store
        const float sx = tx + __shfl_xor(tx, 32, 64), sy = ty + __shfl_xor(ty, 32, 64),
                    sz = tz + __shfl_xor(tz, 32, 64);
        if (valid) {
          if (tx != 0.f || ty != 0.f || tz != 0.f) {
            atomicAdd(&wacc[i * EW + nf + 0], tx);
            atomicAdd(&wacc[i * EW + nf + 1], ty);
            atomicAdd(&wacc[i * EW + nf + 2], tz);
          }
          if (hh == 0) {
            B.colc[Rw * CSTR + NFMAX + 0] = -sx;
            B.colc[Rw * CSTR + NFMAX + 1] = -sy;
            B.colc[Rw * CSTR + NFMAX + 2] = -sz;
          }
        }
      } else if (valid && (tx != 0.f || ty != 0.f || tz != 0.f)) {
        atomicAdd(&wacc[i * EW + nf + 0], tx);
        atomicAdd(&wacc[i * EW + nf + 1], ty);
        atomicAdd(&wacc[i * EW + nf + 2], tz);
        atomicAdd(&wacc[jl * EW + nf + 0], -tx);
        atomicAdd(&wacc[jl * EW + nf + 1], -ty);
        atomicAdd(&wacc[jl * EW + nf + 2], -tz);
      }
    }
    if constexpr (!BIG) break;
    __syncthreads();   // sm.pairs consumed
    if (pp0 + PCAP >= P_all) break;
    }
    __syncthreads();
    for (int e = tid; e < n * EW; e += BLOCK) {
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) s += sm.u.nb[(size_t)ww * n * EW + e];
      const int a = e / EW, q = e - a * EW;
      if (q < nf) sb.ah[a * NFP + q] += s;
      else sb.apos[a * 3 + q - nf] += s;
    }
  }
  __syncthreads();

  STAMP(13);
  // ---- adjoints of the layer input
  for (int e = tid; e < n * 3; e += BLOCK) {
    B.apos[(size_t)a0 * 3 + e] = sb.apos[e];
    B.avel[(size_t)a0 * 3 + e] = sb.avel[e];
  }
  for (int e = tid; e < n * nf; e += BLOCK) {
    const int a = e / nf, q = e - a * nf;
    B.ah[(size_t)a0 * nf + e] = sb.ah[a * NFP + q];
    B.ag[(size_t)a0 * nf + e] = sb.ag[a * NFP + q];
  }
  STAMP(14);
  STAMP_FLUSH
  if (tid == 0 && sm.err) atomicOr(B.err, sm.err);
}

// ---------------------------------------------------------------------------
// per-layer 32-aligned pair row offsets (exclusive scan, one block per layer)
// ---------------------------------------------------------------------------
// A backward whose error word is set leaves NaN in every gradient it produced,
// so an optimizer step that runs before the host reads the (deferred) word
// cannot apply wrong-but-finite updates silently.
__global__ void __launch_bounds__(256) poison_on_err_kernel(const int32_t* __restrict__ err, float* __restrict__ a,
                                                            long long na, float* __restrict__ b, long long nb) {
  if (__builtin_nontemporal_load(err) == 0) return;
  const float nan = __builtin_nanf("");
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < na; i += stride) a[i] = nan;
  if (b)
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += stride) b[i] = nan;
}

__global__ void __launch_bounds__(BLOCK) pair_offsets_kernel(const int32_t* counts, int num_mols, int32_t* offs) {
  __shared__ int wsum[WAVES];
  __shared__ int carry;
  const int l = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int32_t* cnt = counts + (size_t)l * num_mols;
  int32_t* out = offs + (size_t)l * (num_mols + 1);
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < num_mols; base += BLOCK) {
    const int mm = base + tid;
    const int v = mm < num_mols ? ((cnt[mm] + 31) & ~31) : 0;
    const int incl = wave_incl_scan(v);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int pre = carry;
    for (int k = 0; k < w; ++k) pre += wsum[k];
    if (mm < num_mols) out[mm] = pre + incl - v;
    __syncthreads();
    if (tid == BLOCK - 1) carry = pre + incl;
    __syncthreads();
  }
  if (tid == 0) out[num_mols] = carry;
}

// ---------------------------------------------------------------------------
// weight gradients: C[m][n] = sum_rows DY[row][m] X[row][n] (+ bias column
// sum_rows DY[row][m]); rows chunked, one partial per chunk, fixed-order reduce
// ---------------------------------------------------------------------------
struct OuterDesc {
  const float* DY;
  const float* X;
  const int32_t* rows_dev;   // device row count (NULL: rows_static)
  float* part;
  float* outW;               // [M][N] row-major (torch Linear weight layout)
  float* outB;               // [M] (bias) or NULL
  int ldd, M, ldx, N, rows_static, mb, nb, nch;
  int tiled;                 // 0 row-major; 1 tile-blocked (trow layout; ldd / ldx = width);
                             // 2 tile-blocked on the F16X3 kernel (outer_x3_kernel);
                             // 3 partials written by another descriptor's pass (part2)
  int xf_x;                  // 1: X = silu(stored)
  const float* xrow;         // tile-blocked: X[row][n] *= xrow[row] after xf_x (or NULL)
  int xf_dy;                 // 1: DY[row][m] = rowv[row] * colv[m] * silu'(stored)
  const float* rowv;
  const float* colv;
  int chunk;                 // rows per workgroup / partial
  float* part2;              // outer_x3_kernel with xf_dy: partials of sum_rows rowv * silu(DY source)
  int recomp;                // outer_x3_kernel operands recomputed instead of read (RECOMP_*)
  const float* Lp;           // RECOMP_*: the layer's packed forward weights
  int nf;                    // RECOMP_X0: node features (xin row layout)
  const float* actp;         // the layer's act_fn (kind, p0, p1; packed layer + vfl + 1), NULL: SiLU
  int f32r;                  // RECOMP_*: recompute on the fp32 MFMA (the ENFLOW_BWD_F32 backward)
  const float* tmaxA;        // outer_x3_kernel: the producer's per-tile max |DY| / max |X| (BwdArgs::tmax
  const float* tmaxB;        //   + TMX_*, stride TMX_W)
};
// RECOMP_X0: X = silu(pre0), pre0 = edge_nn.0 . xin + be1 (the X source is xin, width ldx);
// RECOMP_PC: DY = rowv * silu'(pc), pc = coord_nn.0 . X + bc1 (X read; no DY source), and
//            part2 gets coord_nn.2's sum_rows rowv * silu(pc).
// Both are the layer backward's instruction sequences on the same operands: bitwise its values.
enum { RECOMP_NONE = 0, RECOMP_X0 = 1, RECOMP_PC = 2 };
#define OUTER_MAX 10
struct OuterBatch {
  OuterDesc d[OUTER_MAX];
  int nd;
  int start[OUTER_MAX + 1];   // first workgroup of each descriptor
};
#ifndef OA_CHUNK
#define OA_CHUNK 2048        // pair rows per partial
#endif
#ifndef OA_CHUNK_ATOM
#define OA_CHUNK_ATOM 256    // atom rows per partial (r04z: 256 -1 % of backward vs 512 on the F16X3 atom-row kernel)
#endif
static_assert(OA_CHUNK % 64 == 0 && OA_CHUNK_ATOM % 64 == 0, "partial chunks are whole row stages");

__device__ __forceinline__ int find_desc(const OuterBatch& ob, int bid) {
  int k = 0;
  while (k + 1 < ob.nd && bid >= ob.start[k + 1]) ++k;
  return k;
}

// One workgroup = one chunk of OA_CHUNK rows x a 128-column block of X, the
// whole M (<= 128) of DY.  Rows are staged through LDS 32 at a time (double
// buffered: the next stage's global loads are in flight during this stage's
// MFMAs).  Waves own 64 x 64 quadrants of the 128 x 128 output as four
// v_mfma_f32_32x32x2_f32 accumulators; each k-step (2 rows) reads its A / B
// fragments straight from the row-major LDS image (lanes along m / n:
// conflict-free).  M == 1 (coord_nn.2 / vel_scaling_nn.2) is a plain column
// reduction and runs on VALU.  The bias column (sum of DY) is accumulated by
// the n-block-0 workgroup from the same LDS image.
#define OB_ROWS 32
#ifndef ENFLOW_ATOM_X3
#define ENFLOW_ATOM_X3 1   // atom-row weight gradients on the F16X3 MFMA (0: fp32 MFMA; A/B knob)
#endif
#ifndef ENFLOW_OUTER_X3
#define ENFLOW_OUTER_X3 1    // pair-row weight gradients on F16X3 MFMA (0: fp32 MFMA)
#endif
#define PAIR_OUTER (ENFLOW_OUTER_X3 ? 2 : 1)
#define OB_LD 129   // LDS row stride: tile-blocked stages write down the columns
template <bool TILED, bool GEN = false>
__global__ void __launch_bounds__(256, 2) outer_acc_kernel(OuterBatch ob) {
  const int bid = blockIdx.x;
  const int k = find_desc(ob, bid);
  const OuterDesc& D = ob.d[k];
  const int local = bid - ob.start[k];
  const int chunk = local / D.nb, nbi = local - chunk * D.nb;
  const int rows = D.rows_dev ? D.rows_dev[0] : D.rows_static;
  const int r0 = chunk * D.chunk;
  if (r0 >= rows) return;
  const int r1 = min(rows, r0 + D.chunk);
  const int NB = D.N + (D.outB ? 1 : 0);
  const int n0 = nbi * 128;
  const int M = D.M, N = D.N;
  const Act act = GEN && D.actp ? act_of(D.actp) : act_silu();
  __shared__ float sd[2][OB_ROWS][OB_LD];
  __shared__ float sx[2][OB_ROWS][OB_LD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, j = lane & 31, hh = lane >> 5;
  const int mh = w & 1, nh = w >> 1;
  const bool do_bias = D.outB != nullptr && nbi == 0 && tid < M;
  float bsum = 0.f;
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (f32x16)0.f;
  float vacc = 0.f;   // M == 1 path: column n0 + tid (tid < 128)
  float rd[16], rx[16];
  const int nst = (r1 - r0 + OB_ROWS - 1) / OB_ROWS;
  constexpr bool tiled = TILED;
  // element q of this thread: (row r, column c) of the 32 x 128 stage; tile-blocked
  // sources are read down the columns (contiguous), row-major ones along the rows
  auto rc = [&](int q, int& r, int& c) {
    const int e = q * 256 + tid;
    if (tiled) { r = e & 31; c = e >> 5; } else { r = e >> 7; c = e & 127; }
  };
  // coord_nn.0's DY = aphi[row] * wc2[m] * silu'(pc): the row factor is applied
  // on load (a thread's 16 elements of a tile-blocked stage share one row), the
  // column factor wc2[m] to the finished sums
  float ra = 0.f, xa = 1.f;
  auto gload = [&](int st) {
    const int rb = r0 + st * OB_ROWS;
    const size_t rt = (size_t)(rb >> 5);
    if (tiled && D.xf_dy) ra = rb + (tid & 31) < r1 ? D.rowv[rb + (tid & 31)] : 0.f;
    if (tiled && D.xrow) xa = rb + (tid & 31) < r1 ? D.xrow[rb + (tid & 31)] : 0.f;
    const float* const dblk = D.DY + ((rt * D.ldd) << 5);            // wave-uniform tile blocks
    const float* const xblk = D.X + ((rt * D.ldx + n0) << 5);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int r, c;
      rc(q, r, c);
      const int p = rb + r;
      const bool pv = p < r1;
      if (tiled) {
        const unsigned e = (unsigned)(q * 256 + tid);                // = c * 32 + r
        rd[q] = (pv && c < M) ? dblk[e] : 0.f;
        rx[q] = (pv && n0 + c < N) ? xblk[e] : 0.f;
      } else {
        rd[q] = (pv && c < M) ? D.DY[(size_t)p * D.ldd + c] : 0.f;
        rx[q] = (pv && n0 + c < N) ? D.X[(size_t)p * D.ldx + n0 + c] : 0.f;
      }
    }
  };
  auto lstore = [&](int buf) {
    if (tiled && D.xf_dy) {
#pragma unroll
      for (int q = 0; q < 16; ++q) rd[q] = ra * dact_v<GEN>(act, rd[q]);
    }
    if (tiled && D.xf_x) {
#pragma unroll
      for (int q = 0; q < 16; ++q) rx[q] = act_v<GEN>(act, rx[q]);
    }
    if (tiled && D.xrow) {
#pragma unroll
      for (int q = 0; q < 16; ++q) rx[q] *= xa;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int r, c;
      rc(q, r, c);
      sd[buf][r][c] = rd[q];
      sx[buf][r][c] = rx[q];
    }
  };
  // wave-uniform: skip accumulator tiles that only see zero padding
  const bool use_m1 = mh * 64 + 32 < M, use_n0 = n0 + nh * 64 < N, use_n1 = n0 + nh * 64 + 32 < N;
  const bool live = mh * 64 < M && use_n0;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) gload(st + 1);
    if (M > 1) {
      if (live && !TILED && ENFLOW_ATOM_X3) {
        // atom rows on the F16X3 MFMA (32x32x16, 3 products) instead of 32x32x2 fp32:
        // each lane gathers its operands' 8 rows per k-step from the row-major stage
        // (A: rows 16 ks + 8 hh + e of DY column m, B: the same rows of X column n),
        // a power-of-two scale per stage, wave and operand (max |x| -> [2^12, 2^13))
        // before the hi / lo split, the stage's sums added with the exact inverse scale
        float av[2][2][8], bv[2][2][8];
        float ma = 0.f, mb = 0.f;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const int r = 16 * ks + 8 * hh + e;
              av[a][ks][e] = sd[buf][r][mh * 64 + a * 32 + j];
              bv[a][ks][e] = sx[buf][r][nh * 64 + a * 32 + j];
              if (a == 0 || use_m1) ma = fmaxf(ma, fabsf(av[a][ks][e]));
              if (a == 0 || use_n1) mb = fmaxf(mb, fabsf(bv[a][ks][e]));
            }
        ma = wave_max(ma);
        mb = wave_max(mb);
        const int ea = pow2_exp(ma), eb = pow2_exp(mb);
        const float sa = ldexpf(1.f, ea), sbs = ldexpf(1.f, eb);
        const float un = ldexpf(ldexpf(1.f, -ea), -eb);
        f16x8 ah[2][2], al[2][2], bh[2][2], bl[2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            f32x16 xa, xb;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              xa[e] = av[a][ks][e] * sa;
              xb[e] = bv[a][ks][e] * sbs;
            }
            split_f16(xa, 0, ah[a][ks], al[a][ks]);
            split_f16(xb, 0, bh[a][ks], bl[a][ks]);
          }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if ((a == 1 && !use_m1) || (b == 1 && !use_n1)) continue;
            f32x16 t = (f32x16)0.f;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
              t = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a][ks], bh[b][ks], t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a][ks], bl[b][ks], t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[a][ks], bh[b][ks], t, 0, 0, 0);
            }
            acc[a][b] += t * un;
          }
      } else if (live) {
        if (use_m1 && use_n1) {
#pragma unroll 4
          for (int s = 0; s < OB_ROWS / 2; ++s) {
            const int r = 2 * s + hh;
            const float a0 = sd[buf][r][mh * 64 + j], a1 = sd[buf][r][mh * 64 + 32 + j];
            const float b0 = sx[buf][r][nh * 64 + j], b1 = sx[buf][r][nh * 64 + 32 + j];
            acc[0][0] = mfma32(a0, b0, acc[0][0]);
            acc[0][1] = mfma32(a0, b1, acc[0][1]);
            acc[1][0] = mfma32(a1, b0, acc[1][0]);
            acc[1][1] = mfma32(a1, b1, acc[1][1]);
          }
        } else {
#pragma unroll 4
          for (int s = 0; s < OB_ROWS / 2; ++s) {
            const int r = 2 * s + hh;
            const float a0 = sd[buf][r][mh * 64 + j], a1 = sd[buf][r][mh * 64 + 32 + j];
            const float b0 = sx[buf][r][nh * 64 + j], b1 = sx[buf][r][nh * 64 + 32 + j];
            acc[0][0] = mfma32(a0, b0, acc[0][0]);
            if (use_n1) acc[0][1] = mfma32(a0, b1, acc[0][1]);
            if (use_m1) acc[1][0] = mfma32(a1, b0, acc[1][0]);
          }
        }
      }
    } else if (tid < 128) {
#pragma unroll 8
      for (int r = 0; r < OB_ROWS; ++r) vacc = fmaf(sd[buf][r][0], sx[buf][r][tid], vacc);
    }
    if (do_bias) {
#pragma unroll 8
      for (int r = 0; r < OB_ROWS; ++r) bsum += sd[buf][r][tid];
    }
    if (st + 1 < nst) lstore(buf ^ 1);
    __syncthreads();
  }
  float* out = D.part + (size_t)chunk * M * NB;
  const bool colf = tiled && D.xf_dy;
  if (M > 1) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mm = mh * 64 + a * 32 + rho(r, hh), nn = n0 + nh * 64 + b * 32 + j;
          if (mm < M && nn < N) out[(size_t)mm * NB + nn] = colf ? acc[a][b][r] * D.colv[mm] : acc[a][b][r];
        }
  } else if (tid < 128 && n0 + tid < N) {
    out[n0 + tid] = vacc;
  }
  if (do_bias) out[(size_t)tid * NB + N] = colf ? bsum * D.colv[tid] : bsum;
}

// F16X3 form of outer_acc_kernel for the tile-blocked pair rows (M > 1): the
// stage's DY / X tiles go to LDS column-major ([column][row], rows contiguous),
// so an MFMA operand (8 consecutive rows of one column) is one ds_read_b128
// pair.  Each operand gets one power-of-two scale per chunk (max |x| of the
// chunk -> [2^12, 2^13), as the layer backward's adjoint tiles) before the
// hi / lo split: the chunk maximum is the max over the per-tile maxima the
// layer backward stored (BwdArgs::tmax), so no stage computes a maximum, the
// three products accumulate straight into acc, and the exact inverse scales
// are applied once to the finished sums.  (Per element the split keeps ~22
// bits relative to the chunk maximum; rows far below it lose low bits that
// the sum could not hold anyway.)
//
// Recomputed operands (OuterDesc::recomp) trade HBM bytes for MFMAs: the layer
// backward stores neither pre(edge_nn.0) nor pre(coord_nn.0) (2 x H floats per
// pair row written and read back), wave w rebuilds output tile w (features
// 32 w .. 32 w + 31) of the stage's 32 rows in the forward's "weights = A"
// orientation (lane = row, registers = features) from the packed forward
// fragments, and writes it to the LDS stage.
#define OX_LD 36   // LDS column stride (floats): 16-byte aligned operand reads
#ifndef ENFLOW_OX_VEC
#define ENFLOW_OX_VEC 1   // 16-B row staging (A/B knob: 0 = one dword per row)
#endif
#ifndef ENFLOW_OUTER_WPS
#define ENFLOW_OUTER_WPS 2   // outer_x3_kernel occupancy hint (A/B knob)
#endif
static_assert(ENFLOW_OUTER_X3 == 1, "pair-row weight gradients run on outer_x3_kernel (recomputed operands)");

// F32R (the ENFLOW_BWD_F32 backward): the recomputed operands come from the
// fp32 MFMA on the forward's fp32 fragments (we1f / wc1f), as that backward's
// own recompute -- an f16x3 split of operands that are entirely small would
// lose the accuracy the fp32 re-run was made for.
template <int H, int RCM, bool GEN = false, bool F32R = false>
__device__ __forceinline__ void outer_x3_body(const OuterDesc& D, int chunk, int nbi, int r0, int r1,
                                              float (*sd)[128][OX_LD], float (*sx)[128][OX_LD]) {
  constexpr int NT = H / 32;
  const int NB = D.N + (D.outB ? 1 : 0);
  const int n0 = nbi * 128;
  const int M = D.M, N = D.N;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hh = lane >> 5;
  const int mh = w & 1, nh = w >> 1;
  constexpr int rcm = RCM;
  const bool do_bias = D.outB != nullptr && nbi == 0 && tid < M;
  const bool xf_dy = D.xf_dy != 0, xf_x = D.xf_x != 0;
  const bool fold = xf_dy && D.part2 != nullptr && nbi == 0;   // coord_nn.2's gradient rides along
  const Act act = GEN && D.actp ? act_of(D.actp) : act_silu();
  // recompute: the layer's packed forward weights
  const int nf = rcm ? D.nf : 1;
  const EgclLayout L = egcl_layout(H, nf);
  const rsrc_t W = weights_rsrc(rcm ? D.Lp : nullptr, rcm ? L.total : 0);
  float wacc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) wacc[q] = 0.f;
  float bsum = 0.f;
  // edge_nn.0's fragments of output tile w (hi / lo per k-step): loop invariant,
  // loaded once per workgroup and kept in registers (RECOMP_X0)
  // (the first k-step's; nf = 8's second k-step is read when used)
  f32x4 wfh = (f32x4)0.f, wfl = (f32x4)0.f;
  if constexpr (rcm == RECOMP_X0 && !F32R) {
    if (w < NT) {
      wfh = bload4(W, lane * 32, (L.we1x + (w * KS0MAX) * 512) * 4);
      wfl = bload4(W, lane * 32 + 16, (L.we1x + (w * KS0MAX) * 512) * 4);
    }
  }
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (f32x16)0.f;
  // staged rows in registers, one stage ahead
  // ENFLOW_OX_VEC: a thread stages 4 consecutive rows of a column per 16-B load /
  // ds_write_b128 (float4 e4 = q * 256 + tid: column e4 / 8, rows 4 (e4 % 8) ..),
  // 4x fewer memory instructions than one dword per row; ra4 / xa4 the 4 rows'
  // factors, raj row j's (the recompute's lane row)
  struct Stage { float rd[16], rx[16], ra, xa; bool pv; f32x4 ra4, xa4; float raj; const float* xb; float rad; };
  Stage S0;
  const int nst = (r1 - r0 + OB_ROWS - 1) / OB_ROWS;
  // thread element q: column c = 8 q + tid / 32, row r = tid % 32 of the stage
  auto gload = [&](int st, Stage& G) {
    const int rb = r0 + st * OB_ROWS;
    const size_t rt = (size_t)(rb >> 5);
    const float* const dblk = D.DY + ((rt * D.ldd) << 5);
    const float* const xblk = D.X + ((rt * D.ldx + n0) << 5);
    const bool pv = rb + (tid & 31) < r1;
    G.pv = pv;
    G.ra = 0.f;
    G.xa = 1.f;
    G.xb = xblk;
#if ENFLOW_OX_VEC
    if (rcm == RECOMP_PC) G.raj = pv ? D.rowv[rb + j] : 0.f;
    if constexpr (rcm != RECOMP_X0) {
      // stage rows are whole 32-row tiles (pair rows are 32-aligned), so a float4
      // of rows is valid or not as a whole
      const int r4 = (tid & 7) * 4;
      const bool pv4 = rb + r4 + 3 < r1;
      G.ra4 = (f32x4)0.f;
      G.xa4 = (f32x4)1.f;
      if (xf_dy) G.ra4 = pv4 ? ld4(D.rowv + rb + r4) : (f32x4)0.f;
      if (D.xrow) G.xa4 = pv4 ? ld4(D.xrow + rb + r4) : (f32x4)0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e4 = q * 256 + tid, c = e4 >> 3;
        f32x4 d = (f32x4)0.f, x = (f32x4)0.f;
        if (rcm != RECOMP_PC && pv4 && c < M) d = ld4(dblk + 4 * e4);
        if (pv4 && n0 + c < N) x = ld4(xblk + 4 * e4);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          G.rd[4 * q + u] = d[u];
          G.rx[4 * q + u] = x[u];
        }
      }
      return;
    } else {   // RECOMP_X0: DY as float4 rows here, the X operand (xin) below
      const int r4 = (tid & 7) * 4;
      const bool pv4 = rb + r4 + 3 < r1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e4 = q * 256 + tid, c = e4 >> 3;
        const f32x4 d = (pv4 && c < M) ? ld4(dblk + 4 * e4) : (f32x4)0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u) G.rd[4 * q + u] = d[u];
      }
    }
#endif
    if (xf_dy) G.ra = pv ? D.rowv[rb + (tid & 31)] : 0.f;
    if (D.xrow) G.xa = pv ? D.xrow[rb + (tid & 31)] : 0.f;
    if constexpr (rcm != RECOMP_PC && !ENFLOW_OX_VEC) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int c = 8 * q + (tid >> 5);
        G.rd[q] = (pv && c < M) ? dblk[(unsigned)(q * 256 + tid)] : 0.f;
      }
    }
    if constexpr (rcm == RECOMP_X0 && F32R) {
      // the fp32 GEMM0 reads its operands from the xin rows in lstore (G.xb)
    } else if constexpr (rcm == RECOMP_X0) {
      // GEMM0's B operand of lane (row j, half hh), as the layer backward builds it
      // (k order gemm0_col): rx[8 ks + u] = k-slice ks, half 0 = h_i's features
      // 8 ks + u, half 1 = h_j's (+ radial in slot 7 of the last slice when that is
      // padding); nf = 8: rx[8] = radial (the second k-slice)
      if constexpr (NFMAX == 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int q = hh ? nf + u : u;
          G.rx[u] = (pv && u < nf) ? xblk[q * 32 + j] : 0.f;
        }
        if (hh && nf <= 7) G.rx[7] = pv ? xblk[(2 * nf) * 32 + j] : 0.f;
        G.rx[8] = pv ? xblk[(2 * nf) * 32 + j] : 0.f;
      } else {   // features in two k-slices; nf 8 / 16: the radial in a slice of its own
        const int nch = gemm0_nch(nf);
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int f = u, q = hh ? nf + f : f;
          G.rx[u] = (pv && f < nf && u < 8 * nch) ? xblk[q * 32 + j] : 0.f;
        }
        const float rad = pv ? xblk[(2 * nf) * 32 + j] : 0.f;
        G.rad = 0.f;
        if (gemm0_radial_slot7(nf)) {
          if (hh) {   // slot 8 nch - 1 (nch 1 / 2), by compile-time index: a runtime one puts Stage in scratch
#pragma unroll
            for (int u = 7; u < 16; u += 8)
              if (u == 8 * nch - 1) G.rx[u] = rad;
          }
        } else if (hh == 0) {
          if (nch == 1) G.rx[8] = rad;   // nf == 8: the radial's own (second) slice
          else G.rad = rad;              // nf == 16: the third slice
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int c = 8 * q + (tid >> 5);
        G.rx[q] = (pv && n0 + c < N) ? xblk[(unsigned)(q * 256 + tid)] : 0.f;
      }
    }
  };
  auto lstore = [&](int buf, Stage& G) {
#if ENFLOW_OX_VEC
    if constexpr (rcm != RECOMP_X0) {
      const int r4 = (tid & 7) * 4;
      if constexpr (rcm != RECOMP_PC) {
        if (xf_dy) {   // DY = aphi * silu'(pc) (wc2 applied at the end); d wc2 += aphi * silu(pc)
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const float z = G.rd[4 * q + u];
              float fz, dz;
              act_fd<GEN>(act, z, fz, dz);
              if (fold) wacc[q] = fmaf(G.ra4[u], fz, wacc[q]);
              G.rd[4 * q + u] = G.ra4[u] * dz;
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          st4(&sd[buf][(q * 256 + tid) >> 3][r4],
              (f32x4){G.rd[4 * q], G.rd[4 * q + 1], G.rd[4 * q + 2], G.rd[4 * q + 3]});
      }
      if (xf_x) {
#pragma unroll
        for (int q = 0; q < 16; ++q) G.rx[q] = act_v<GEN>(act, G.rx[q]);
      }
      if (D.xrow) {
#pragma unroll
        for (int q = 0; q < 16; ++q) G.rx[q] *= G.xa4[q & 3];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st4(&sx[buf][(q * 256 + tid) >> 3][r4], (f32x4){G.rx[4 * q], G.rx[4 * q + 1], G.rx[4 * q + 2], G.rx[4 * q + 3]});
      return;
    } else {   // RECOMP_X0: DY rows as float4 (no transform on edge_nn.2's DY)
      const int r4 = (tid & 7) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st4(&sd[buf][(q * 256 + tid) >> 3][r4],
            (f32x4){G.rd[4 * q], G.rd[4 * q + 1], G.rd[4 * q + 2], G.rd[4 * q + 3]});
    }
#endif
    if constexpr (rcm != RECOMP_PC && !(ENFLOW_OX_VEC && rcm == RECOMP_X0)) {
      if (xf_dy) {   // DY = aphi * silu'(pc) (wc2 applied at the end); d wc2 += aphi * silu(pc)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const float z = G.rd[q];
          float fz, dz;
          act_fd<GEN>(act, z, fz, dz);
          if (fold) wacc[q] = fmaf(G.ra, fz, wacc[q]);
          G.rd[q] = G.ra * dz;
        }
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) sd[buf][8 * q + (tid >> 5)][tid & 31] = G.rd[q];
    }
    if constexpr (rcm == RECOMP_X0 && F32R) {
      if (w < NT) {   // output tile w of pre0 -> act -> X, fp32 MFMA (the forward's f32 GEMM0 k order)
        f32x16 x = (f32x16)0.f;
#pragma unroll
        for (int s = 0; s < NFMAX + 1; ++s) {
          int col = -1;
          if (s < NFMAX / 2) {
            const int f = 2 * s + hh;
            if (f < nf) col = f;
          } else if (s < NFMAX) {
            const int f = 2 * (s - NFMAX / 2) + hh;
            if (f < nf) col = nf + f;
          } else if (hh == 0) {
            col = 2 * nf;
          }
          const float b = (G.pv && col >= 0) ? G.xb[col * 32 + j] : 0.f;
          x = mfma32(bload(W, lane * 4, (L.we1f + (w * (NFMAX + 1) + s) * 64) * 4), b, x);
        }
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int f0 = 32 * w + 8 * g4 + 4 * hh;
          const f32x4 b = ld4(D.Lp + L.be1 + f0);
#pragma unroll
          for (int u = 0; u < 4; ++u) sx[buf][f0 + u][j] = G.pv ? act_v<GEN>(act, x[4 * g4 + u] + b[u]) : 0.f;
        }
      }
    } else if constexpr (rcm == RECOMP_X0) {
      if (w < NT) {   // output tile w of pre0 -> silu -> X
        const int ks_n = gemm0_ksteps(nf);
        f32x16 x = (f32x16)0.f;
        for (int ks = 0; ks < ks_n; ++ks) {
          f32x16 in;
          if constexpr (NFMAX == 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) in[u] = ks == 0 ? G.rx[u] : 0.f;
            if (ks == 1 && hh == 0) in[0] = G.rx[8];
          } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) in[u] = ks == 0 ? G.rx[u] : (ks == 1 ? G.rx[8 + u] : 0.f);
            if (ks == 2) in[0] = G.rad;   // nf 16's radial slice (0 on lane half 1)
          }
          f16x8 bh, bl;
          split_f16(in, 0, bh, bl);
          f32x4 ah = wfh, al = wfl;
          if (ks >= 1) {
            ah = bload4(W, lane * 32, (L.we1x + (w * KS0MAX + ks) * 512) * 4);
            al = bload4(W, lane * 32 + 16, (L.we1x + (w * KS0MAX + ks) * 512) * 4);
          }
          x = mfma_f16(ah, bh, x);
          x = mfma_f16(ah, bl, x);
          x = mfma_f16(al, bh, x);
        }
        x *= D.Lp[L.scl + 5];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int f0 = 32 * w + 8 * g4 + 4 * hh;
          const f32x4 b = ld4(D.Lp + L.be1 + f0);
#pragma unroll
          for (int u = 0; u < 4; ++u) sx[buf][f0 + u][j] = G.pv ? act_v<GEN>(act, x[4 * g4 + u] + b[u]) : 0.f;
        }
      }
    } else {
      if (xf_x) {
#pragma unroll
        for (int q = 0; q < 16; ++q) G.rx[q] = act_v<GEN>(act, G.rx[q]);
      }
      if (D.xrow) {
#pragma unroll
        for (int q = 0; q < 16; ++q) G.rx[q] *= G.xa;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) sx[buf][8 * q + (tid >> 5)][tid & 31] = G.rx[q];
    }
  };
  // RECOMP_PC, after the stage's X is in LDS: pc = coord_nn.0 . X + bc1 (output
  // tile w), DY = aphi * silu'(pc) into LDS, d wc2 partial += aphi * silu(pc)
  float (&wacc2)[16] = wacc;   // RECOMP_PC's d wc2 partials (lane = row, registers = features)
  auto recomp_pc = [&](int buf, const Stage& G) {
    if (F32R && w < NT) {   // fp32 chain of output tile w on wc1f (the forward's f32 k order)
      f32x16 cacc = (f32x16)0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x16 X;
#pragma unroll
        for (int r = 0; r < 16; ++r) X[r] = sx[buf][32 * t + rho(r, hh)][j];
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          const f32x4 a4 = bload4(W, lane * 16, (L.wc1f + ((w * NT + t) * 4 + rg) * 256) * 4);
#pragma unroll
          for (int u = 0; u < 4; ++u) cacc = mfma32(a4[u], X[4 * rg + u], cacc);
        }
      }
      const float ra = ENFLOW_OX_VEC ? G.raj : G.ra;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int f0 = 32 * w + 8 * g4 + 4 * hh;
        const f32x4 b = ld4(D.Lp + L.bc1 + f0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float z = cacc[4 * g4 + u] + b[u];
          float fz, dz;
          act_fd<GEN>(act, z, fz, dz);
          wacc2[4 * g4 + u] = fmaf(ra, fz, wacc2[4 * g4 + u]);
          sd[buf][f0 + u][j] = ra * dz;
        }
      }
    } else if (w < NT) {
      // coord_nn.0's fragments of output tile w, requested half a chain at a time
      // (two L2 round trips per stage; resident they would cost 64 VGPRs across
      // the stage)
      constexpr int HALF = NT > 1 ? NT : 2;   // k-steps per request group
      f32x16 cacc = (f32x16)0.f;
#pragma unroll
      for (int g = 0; g < 2 * NT; g += HALF) {
        f32x4 ch[HALF], cl[HALF];
#pragma unroll
        for (int q = 0; q < HALF; ++q) {
          const int ts = g + q;
          const int so = (L.wc1x + ((w * NT + (ts >> 1)) * 2 + (ts & 1)) * 512) * 4;
          ch[q] = bload4(W, lane * 32, so);
          cl[q] = bload4(W, lane * 32 + 16, so);
        }
        // chain_x3_fill's per-tile order: k-steps ascending, hi.hi, hi.lo, lo.hi
#pragma unroll
        for (int q = 0; q < HALF; q += 2) {
          const int t = (g + q) >> 1;
          f32x16 X;   // input tile t in the accumulator layout (lane = row, registers = features)
#pragma unroll
          for (int r = 0; r < 16; ++r) X[r] = sx[buf][32 * t + rho(r, hh)][j];
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            f16x8 bh, bl;
            split_f16(X, s2, bh, bl);
            cacc = mfma_f16(ch[q + s2], bh, cacc);
            cacc = mfma_f16(ch[q + s2], bl, cacc);
            cacc = mfma_f16(cl[q + s2], bh, cacc);
          }
        }
      }
      const float inv2 = D.Lp[L.scl + 3];
      const float ra = ENFLOW_OX_VEC ? G.raj : G.ra;   // row j's aphi
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int f0 = 32 * w + 8 * g4 + 4 * hh;
        const f32x4 b = ld4(D.Lp + L.bc1 + f0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float z = fmaf(cacc[4 * g4 + u], inv2, b[u]);
          float fz, dz;
          act_fd<GEN>(act, z, fz, dz);
          wacc2[4 * g4 + u] = fmaf(ra, fz, wacc2[4 * g4 + u]);
          sd[buf][f0 + u][j] = ra * dz;
        }
      }
    }
  };
  const bool use_m1 = mh * 64 + 32 < M, use_n0 = n0 + nh * 64 < N, use_n1 = n0 + nh * 64 + 32 < N;
  const bool live = mh * 64 < M && use_n0;
  // the chunk's scales (one per operand, from the producer's per-tile maxima):
  // max |x| of the chunk -> [2^12, 2^13) before the hi / lo split, so the three
  // products accumulate straight into acc and are un-scaled once at the end
  static_assert(OA_CHUNK <= 64 * 32, "a chunk's tile maxima fit one wave");
  int ea = 0, eb = 0;
  {
    const int t0 = r0 >> 5, ntl = (r1 - r0 + 31) >> 5;
    const float ma = lane < ntl ? D.tmaxA[(size_t)(t0 + lane) * TMX_W] : 0.f;
    const float mb = lane < ntl ? D.tmaxB[(size_t)(t0 + lane) * TMX_W] : 0.f;
    ea = pow2_exp(wave_max(ma));
    eb = pow2_exp(wave_max(mb));
  }
  const float sa = ldexpf(1.f, ea), sbs = ldexpf(1.f, eb);
  auto compute = [&](int buf) {
    if (live) {
      // operands of both k-steps: A[a][ks] (DY columns), B[b][ks] (X columns)
      f32x4 av[2][2][2], bv[2][2][2];   // [tile][ks][half]
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            av[a][ks][h2] = *reinterpret_cast<const f32x4*>(&sd[buf][mh * 64 + a * 32 + j][16 * ks + 8 * hh + 4 * h2]);
            bv[a][ks][h2] = *reinterpret_cast<const f32x4*>(&sx[buf][nh * 64 + a * 32 + j][16 * ks + 8 * hh + 4 * h2]);
          }
      f16x8 ah[2][2], al[2][2], bh[2][2], bl[2][2];
      // scaled hi / lo split: hi = f16(x s) by v_cvt_pk_f16_f32, lo = f16(x s - hi) by
      // v_fma_mix (split_f16; x s - hi is exact in fp32, so bitwise the plain form)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          f32x16 xa, xb;
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            xa[jj] = av[a][ks][jj >> 2][jj & 3] * sa;
            xb[jj] = bv[a][ks][jj >> 2][jj & 3] * sbs;
          }
          split_f16(xa, 0, ah[a][ks], al[a][ks]);
          split_f16(xb, 0, bh[a][ks], bl[a][ks]);
        }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          if ((a == 1 && !use_m1) || (b == 1 && !use_n1)) continue;
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a][ks], bh[b][ks], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[a][ks], bl[b][ks], acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[a][ks], bh[b][ks], acc[a][b], 0, 0, 0);
          }
        }
    }
    if (do_bias) {
#pragma unroll 8
      for (int r = 0; r < OB_ROWS; ++r) bsum += sd[buf][tid][r];
    }
  };
  gload(0, S0);
  lstore(0, S0);
  __syncthreads();
  if constexpr (rcm == RECOMP_PC) {
    recomp_pc(0, S0);
    __syncthreads();
  }
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) gload(st + 1, S0);
    compute(buf);
    if (st + 1 < nst) lstore(buf ^ 1, S0);
    __syncthreads();
    if (rcm == RECOMP_PC && st + 1 < nst) {
      recomp_pc(buf ^ 1, S0);
      __syncthreads();
    }
  }
  float* out = D.part + (size_t)chunk * M * NB;
  const float ua = ldexpf(1.f, -ea), ub = ldexpf(1.f, -eb);   // exact inverse scales
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = mh * 64 + a * 32 + rho(r, hh), nn = n0 + nh * 64 + b * 32 + j;
        const float v = acc[a][b][r] * ua * ub;
        if (mm < M && nn < N) out[(size_t)mm * NB + nn] = xf_dy ? v * D.colv[mm] : v;
      }
  if (do_bias) out[(size_t)tid * NB + N] = xf_dy ? bsum * D.colv[tid] : bsum;
  if (fold && rcm == RECOMP_PC) {   // fixed-order sum over the 32 rows of each half-wave
    if (w < NT) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = wacc2[r];
#pragma unroll
        for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (j == 0) D.part2[(size_t)chunk * M + 32 * w + rho(r, hh)] = v;
      }
    }
  } else if (fold && ENFLOW_OX_VEC) {   // fixed-order sum over the 8 row groups of each column
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = wacc[q];
#pragma unroll
      for (int off = 1; off < 8; off <<= 1) v += __shfl_xor(v, off, 64);
      const int c = (q * 256 + tid) >> 3;
      if ((tid & 7) == 0 && c < M) D.part2[(size_t)chunk * M + c] = v;
    }
  } else if (fold) {   // fixed-order sum over the 32 rows a half-wave holds
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float v = wacc[q];
#pragma unroll
      for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
      if ((tid & 31) == 0 && 8 * q + (tid >> 5) < M) D.part2[(size_t)chunk * M + 8 * q + (tid >> 5)] = v;
    }
  }
}

template <bool GEN = false, bool F32R = false>
__global__ void __launch_bounds__(256, ENFLOW_OUTER_WPS) outer_x3_kernel(OuterBatch ob) {
  const int bid = blockIdx.x;
  const int k = find_desc(ob, bid);
  const OuterDesc& D = ob.d[k];
  const int local = bid - ob.start[k];
  const int chunk = local / D.nb, nbi = local - chunk * D.nb;
  const int rows = D.rows_dev ? D.rows_dev[0] : D.rows_static;
  const int r0 = chunk * D.chunk;
  if (r0 >= rows) return;
  const int r1 = min(rows, r0 + D.chunk);
  __shared__ float sd[2][128][OX_LD];
  __shared__ float sx[2][128][OX_LD];
  // recomputed operands need the layer's hidden width at compile time
  // (one register allocation per branch: the modes' staged operands differ)
  if (D.recomp == RECOMP_X0) {
    if (D.N == 128) outer_x3_body<128, RECOMP_X0, GEN, F32R>(D, chunk, nbi, r0, r1, sd, sx);
    else if (D.N == 64) outer_x3_body<64, RECOMP_X0, GEN, F32R>(D, chunk, nbi, r0, r1, sd, sx);
    else outer_x3_body<32, RECOMP_X0, GEN, F32R>(D, chunk, nbi, r0, r1, sd, sx);
  } else if (D.recomp == RECOMP_PC) {
    if (D.N == 128) outer_x3_body<128, RECOMP_PC, GEN, F32R>(D, chunk, nbi, r0, r1, sd, sx);
    else if (D.N == 64) outer_x3_body<64, RECOMP_PC, GEN, F32R>(D, chunk, nbi, r0, r1, sd, sx);
    else outer_x3_body<32, RECOMP_PC, GEN, F32R>(D, chunk, nbi, r0, r1, sd, sx);
  } else {
    outer_x3_body<128, RECOMP_NONE, GEN>(D, chunk, nbi, r0, r1, sd, sx);
  }
}

// Four fp64 sums per output (chunk mod 4, the leftover chunks into the first),
// one per thread of a 4-lane group, combined in the fixed order (s0 + s1) +
// (s2 + s3): 64 outputs per workgroup, so the partials stream through 4x as
// many workgroups with a quarter of the serial loads each
#define RP_OUT 64
__global__ void __launch_bounds__(256) reduce_part_kernel(OuterBatch ob) {
  const int bid = blockIdx.x;
  const int k = find_desc(ob, bid);
  const OuterDesc& D = ob.d[k];
  const int rows = D.rows_dev ? D.rows_dev[0] : D.rows_static;
  const int nch = (rows + D.chunk - 1) / D.chunk;
  const int NB = D.N + (D.outB ? 1 : 0);
  const int sub = threadIdx.x & 3;
  const int idx = (bid - ob.start[k]) * RP_OUT + (threadIdx.x >> 2);
  const bool live = idx < D.M * NB;   // (the whole 4-lane group agrees)
  const size_t cs = (size_t)D.M * NB;
  const float* src = D.part + (live ? idx : 0);
  double s = 0.0;
  const int G = nch >> 2;
  if (live) {
    // eight chunk groups per step into independent sums (eight loads in flight
    // per lane; the partials are read once: non-temporal), combined in a fixed
    // order: deterministic
    constexpr int U = 8;
    double su[U];
#pragma unroll
    for (int u = 0; u < U; ++u) su[u] = 0.0;
    int g = 0;
    for (; g + U <= G; g += U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(&src[(size_t)(4 * (g + u) + sub) * cs]);
#pragma unroll
      for (int u = 0; u < U; ++u) su[u] += (double)v[u];
    }
    for (; g < G; ++g) su[0] += (double)__builtin_nontemporal_load(&src[(size_t)(4 * g + sub) * cs]);
    s = ((su[0] + su[1]) + (su[2] + su[3])) + ((su[4] + su[5]) + (su[6] + su[7]));
    if (sub == 0)
      for (int ch = 4 * G; ch < nch; ++ch) s += (double)src[(size_t)ch * cs];
  }
  const double pair = s + __shfl_xor(s, 1, 64);      // lane 0: s0 + s1, lane 2: s2 + s3
  const double tot = pair + __shfl_xor(pair, 2, 64);  // lane 0: (s0 + s1) + (s2 + s3)
  if (!live || sub != 0) return;
  const int mm = idx / NB, nn = idx - mm * NB;
  if (nn < D.N) D.outW[(size_t)mm * D.N + nn] = (float)tot;
  else D.outB[mm] = (float)tot;
}

// ---------------------------------------------------------------------------
// ArgMax.forward backward (enflow/nn/argmax.py:13-25): adjoint of z (= d h at
// the first layer's input) and of log_q (= d ldj) -> parameter-gradient rows
// ---------------------------------------------------------------------------
template <int H, int NMAX>
__global__ void __launch_bounds__(BLOCK) argmax_bwd_kernel(const int32_t* mol_ptr, int nf, const float* hdata,
                                                          const float* noise, const float* Draw, const float* az,
                                                          const float* adj_ldj, float* apre_rows, float* spre_rows,
                                                          float* anet_rows) {
  __shared__ float pre[NMAX][H + 1];
  __shared__ float spv[NMAX][H + 1];   // act(pre), once per (atom, unit): network.2's input
  __shared__ float net[NMAX][2 * NFMAX];
  __shared__ float anet[NMAX][2 * NFMAX];
  __shared__ float hs[NMAX][NFMAX];
  const int m = blockIdx.x, tid = threadIdx.x;
  const int a0 = mol_ptr[m], n = mol_ptr[m + 1] - a0;
  if (n > NMAX) return;
  const int rW1 = 0, rb1 = H * nf, rW2 = rb1 + H, rb2 = rW2 + 2 * nf * H;
  const Act am = act_of(Draw + rb2 + 2 * nf);   // network.1 (the raw vector's act trailer, ABI 10)
  for (int e = tid; e < n * nf; e += BLOCK) hs[e / nf][e % nf] = hdata[(size_t)a0 * nf + e];
  __syncthreads();
  constexpr int NG = BLOCK / H;
  const int k = tid % H, grp = tid / H;
  for (int a = grp; a < n; a += NG) {
    float v = Draw[rb1 + k];
    for (int f = 0; f < nf; ++f) v = fmaf(Draw[rW1 + k * nf + f], hs[a][f], v);
    pre[a][k] = v;
    const float sv = am.k == ACT_SILU ? v * sigmoid_f(v) : act_f(am, v);
    spv[a][k] = sv;
    spre_rows[(size_t)(a0 + a) * H + k] = sv;
  }
  __syncthreads();
  for (int e = tid; e < n * 2 * nf; e += BLOCK) {
    const int a = e / (2 * nf), o = e - a * 2 * nf;
    float s = Draw[rb2 + o];
    for (int kk = 0; kk < H; ++kk) s = fmaf(Draw[rW2 + o * H + kk], spv[a][kk], s);
    net[a][o] = s;
  }
  __syncthreads();
  const float aldj = adj_ldj[0];
  if (tid < n) {
    const int a = tid;
    float u[NFMAX], hv[NFMAX], sg[NFMAX], zz[NFMAX], els[NFMAX];
    float T = 0.f;
#pragma unroll
    for (int q = 0; q < NFMAX; ++q) {
      if (q < nf) {
        els[q] = expf(net[a][q]);
        u[q] = net[a][nf + q] + noise[(size_t)(a0 + a) * nf + q] * els[q];
        hv[q] = hs[a][q];
        zz[q] = az[(size_t)(a0 + a) * nf + q];
        T += hv[q] * u[q];
      }
    }
    float S = 0.f, Az = 0.f;
#pragma unroll
    for (int q = 0; q < NFMAX; ++q) {
      if (q < nf) {
        sg[q] = sigmoid_f(T - u[q]);
        const float w = (1.f - hv[q]) * (1.f - sg[q]);
        S += w;
        Az += zz[q] * w;
      }
    }
#pragma unroll
    for (int q = 0; q < NFMAX; ++q) {
      if (q < nf) {
        const float au = zz[q] * hv[q] + (1.f - hv[q]) * zz[q] * sg[q] + hv[q] * Az +
                         aldj * (-u[q] - hv[q] * S + (1.f - hv[q]) * (1.f - sg[q]));
        const float als = au * noise[(size_t)(a0 + a) * nf + q] * els[q] - aldj;
        anet[a][q] = als;
        anet[a][nf + q] = au;
        anet_rows[(size_t)(a0 + a) * 2 * nf + q] = als;
        anet_rows[(size_t)(a0 + a) * 2 * nf + nf + q] = au;
      }
    }
  }
  __syncthreads();
  for (int a = grp; a < n; a += NG) {
    float s = 0.f;
    for (int o = 0; o < 2 * nf; ++o) s = fmaf(Draw[rW2 + o * H + k], anet[a][o], s);
    const float p = pre[a][k];
    if (am.k == ACT_SILU) {
      const float sp = sigmoid_f(p);
      apre_rows[(size_t)(a0 + a) * H + k] = s * sp * (1.f + p * (1.f - sp));
    } else {
      apre_rows[(size_t)(a0 + a) * H + k] = s * act_d(am, p);
    }
  }
}

// ---------------------------------------------------------------------------
// Alchemical_NLL backward (enflow/flow/loss.py:11-24)
// ---------------------------------------------------------------------------
template <int NMAX>
__global__ void __launch_bounds__(BLOCK) nll_bwd_kernel(const int32_t* mol_ptr, int num_mols, int nf, const float* h,
                                                      const float* g, const float* pos, const float* vel, float kBT,
                                                      float softening, const float* grad_loss, float* ah, float* ag,
                                                      float* apos, float* avel, float* adj_ldj) {
  __shared__ float spos[NMAX * 3];
  const int m = blockIdx.x, tid = threadIdx.x;
  const int a0 = mol_ptr[m], n = mol_ptr[m + 1] - a0;
  const float s = grad_loss ? grad_loss[0] : 1.f;
  const float invM = s / (float)num_mols;
  const float cH = invM / kBT;
  for (int e = tid; e < n * 3; e += BLOCK) {
    spos[e] = pos[(size_t)a0 * 3 + e];
    avel[(size_t)a0 * 3 + e] = cH * vel[(size_t)a0 * 3 + e];    // H = LJ + 0.5 vel^2
  }
  for (int e = tid; e < n * nf; e += BLOCK) {                    // -log_gaussian(h), (g)
    ah[(size_t)a0 * nf + e] = invM * h[(size_t)a0 * nf + e];
    ag[(size_t)a0 * nf + e] = invM * g[(size_t)a0 * nf + e];
  }
  __syncthreads();
  for (int e = tid; e < n * 3; e += BLOCK) {
    const int a = e / 3, d = e - a * 3;
    float f = 0.f;
    for (int b = 0; b < n; ++b) {
      if (b == a) continue;
      const float dx = spos[a * 3] - spos[b * 3], dy = spos[a * 3 + 1] - spos[b * 3 + 1],
                  dz = spos[a * 3 + 2] - spos[b * 3 + 2];
      const float d2 = dx * dx + dy * dy + dz * dz;
      if (d2 == 0.f) continue;                                   // dist_sq != 0 (loss.py:15)
      const float r = d2 + softening, ir = 1.f / r, ir2 = ir * ir, ir4 = ir2 * ir2;
      const float dEdR = 4.f * (-6.f * ir4 * ir2 * ir + 3.f * ir4);
      f += dEdR * 2.f * (spos[a * 3 + d] - spos[b * 3 + d]);
    }
    apos[(size_t)a0 * 3 + e] = cH * f;
  }
  if (m == 0 && tid == 0) adj_ldj[0] = -invM;                    // log_px += ldj
}

// ---------------------------------------------------------------------------
// large systems: pair-row offsets of the row blocks, column-side adjoint sums
// ---------------------------------------------------------------------------
// one workgroup: boff[b] = 32-aligned exclusive prefix of the blocks' pair words,
// total[0] = all rows (the weight-gradient passes' row count)
__device__ __forceinline__ int lg_block_words(const int32_t* mol_ptr, int num_mols, const int32_t* blk_start,
                                              int rbl, const int32_t* npairs, int b) {
  const int m = seg_of(blk_start, num_mols, b);
  const int a0 = mol_ptr[m], n = mol_ptr[m + 1] - a0;
  const int r0 = (b - blk_start[m]) * rbl, rb = min(rbl, n - r0);
  int t = 0;
  for (int a = 0; a < rb; ++a) t += npairs[a0 + r0 + a];
  return (t + 31) & ~31;
}
__global__ void __launch_bounds__(BLOCK) lg_bwd_offsets_kernel(const int32_t* mol_ptr, int num_mols,
                                                               const int32_t* blk_start, int rbl,
                                                               const int32_t* npairs, int32_t* boff,
                                                               int32_t* total) {
  __shared__ int part[BLOCK + 1];
  const int tid = threadIdx.x;
  const int nb = blk_start[num_mols];
  const int per = (nb + BLOCK - 1) / BLOCK;
  const int b0 = min(nb, tid * per), b1 = min(nb, b0 + per);
  int s = 0;
  for (int b = b0; b < b1; ++b) s += lg_block_words(mol_ptr, num_mols, blk_start, rbl, npairs, b);
  part[tid] = s;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int k = 0; k < BLOCK; ++k) { const int v = part[k]; part[k] = acc; acc += v; }
    part[BLOCK] = acc;
    total[0] = acc;
  }
  __syncthreads();
  int acc = part[tid];
  for (int b = b0; b < b1; ++b) {
    boff[b] = acc;
    acc += lg_block_words(mol_ptr, num_mols, blk_start, rbl, npairs, b);
  }
}

// partial column sums: thread = column atom q of its molecule, blockIdx.y = a
// chunk of LG_RC rows; the rows' slots of q (smap, coalesced over q) locate the
// pair's column adjoints in colc; rows in increasing order -> deterministic
constexpr int LG_RC = 64;
__global__ void __launch_bounds__(BLOCK) lg_colsum_kernel(const int32_t* mol_ptr, int num_mols, int num_atoms,
                                                          int max_n, const int32_t* smap, const int32_t* rowstart,
                                                          const float* colc, int nf, float* part) {
  const int q = blockIdx.x * BLOCK + threadIdx.x, ch = blockIdx.y;
  if (q >= num_atoms) return;
  const int m = seg_of(mol_ptr, num_mols, q);
  const int a0 = mol_ptr[m], n = mol_ptr[m + 1] - a0, ql = q - a0;
  const int i0 = min(n, ch * LG_RC), i1 = min(n, i0 + LG_RC);
  float acc[NFMAX + 3];
#pragma unroll
  for (int k = 0; k < NFMAX + 3; ++k) acc[k] = 0.f;
  for (int i = i0; i < i1; ++i) {
    const int k = smap[(size_t)(a0 + i) * max_n + ql];
    if (k >= 0) {
      const float* c = colc + (size_t)(rowstart[a0 + i] + k) * CSTR;
      for (int f = 0; f < nf; ++f) acc[f] += c[f];
#pragma unroll
      for (int d = 0; d < 3; ++d) acc[NFMAX + d] += c[NFMAX + d];
    }
  }
  float* o = part + ((size_t)ch * num_atoms + q) * CSTR;
#pragma unroll
  for (int k = 0; k < NFMAX + 3; ++k) o[k] = acc[k];
}

// column label c = id_mapping[q] (base.py:137): atom c receives the column sums
// of every q mapped to it, q and chunks in increasing order.  One wave per label:
// the lanes test 64 q at a time, the matches are taken in q order (ballot bits),
// lane k < nf + 3 sums component k
__global__ void __launch_bounds__(BLOCK) lg_colfinal_kernel(const int32_t* mol_ptr, int num_mols, int num_atoms,
                                                            const int32_t* idmap, const float* part, int nch,
                                                            int nf, float* ah, float* apos) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (c >= num_atoms) return;   // wave-uniform
  const int m = seg_of(mol_ptr, num_mols, c);
  const int a0 = mol_ptr[m], n = mol_ptr[m + 1] - a0, cl = c - a0;
  const int comp = lane < nf ? lane : (lane >= NFMAX && lane < NFMAX + 3 ? lane : -1);
  float acc = 0.f;
  for (int q0 = 0; q0 < n; q0 += 64) {
    const int q = q0 + lane;
    uint64_t hit = __ballot(q < n && idmap[a0 + q] == cl);
    while (hit) {   // wave-uniform loop over the matches, lowest q first
      const int qq = q0 + __builtin_ctzll(hit);
      hit &= hit - 1;
      if (comp >= 0)
        for (int ch = 0; ch < nch; ++ch) acc += part[((size_t)ch * num_atoms + a0 + qq) * CSTR + comp];
    }
  }
  if (lane < nf) ah[(size_t)c * nf + lane] += acc;
  else if (comp >= 0) apos[(size_t)c * 3 + (lane - NFMAX)] += acc;
}

// atom chunks of <= 32 for the per-atom ArgMax backward on large systems
__global__ void __launch_bounds__(BLOCK) chunk_ptr_kernel(int num_atoms, int chunks, int32_t* ptr) {
  const int k = blockIdx.x * BLOCK + threadIdx.x;
  if (k <= chunks) ptr[k] = min(32 * k, num_atoms);
}

// Alchemical_NLL backward for molecules past 64 atoms: one wave per atom (lanes
// over the molecule's other atoms, fixed butterfly reduction), positions from L2
__global__ void __launch_bounds__(BLOCK) nll_bwd_large_kernel(const int32_t* mol_ptr, int num_mols, int num_atoms,
                                                              int nf, const float* h, const float* g,
                                                              const float* pos, const float* vel, float kBT,
                                                              float softening, const float* grad_loss, float* ah,
                                                              float* ag, float* apos, float* avel,
                                                              float* adj_ldj) {
  const int lane = threadIdx.x & 63;
  const int a = blockIdx.x * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const float s = grad_loss ? grad_loss[0] : 1.f;
  const float invM = s / (float)num_mols;
  const float cH = invM / kBT;
  if (a == 0 && lane == 0) adj_ldj[0] = -invM;                   // log_px += ldj
  if (a >= num_atoms) return;                                    // wave-uniform
  const int m = seg_of(mol_ptr, num_mols, a);
  const int a0 = mol_ptr[m], n = mol_ptr[m + 1] - a0;
  if (lane < 3) avel[(size_t)a * 3 + lane] = cH * vel[(size_t)a * 3 + lane];   // H = LJ + 0.5 vel^2
  if (lane < nf) {                                               // -log_gaussian(h), (g)
    ah[(size_t)a * nf + lane] = invM * h[(size_t)a * nf + lane];
    ag[(size_t)a * nf + lane] = invM * g[(size_t)a * nf + lane];
  }
  const float px = pos[(size_t)a * 3], py = pos[(size_t)a * 3 + 1], pz = pos[(size_t)a * 3 + 2];
  float fx = 0.f, fy = 0.f, fz = 0.f;
  for (int b = a0 + lane; b < a0 + n; b += 64) {
    if (b == a) continue;
    const float dx = px - pos[(size_t)b * 3], dy = py - pos[(size_t)b * 3 + 1], dz = pz - pos[(size_t)b * 3 + 2];
    const float d2 = dx * dx + dy * dy + dz * dz;
    if (d2 == 0.f) continue;                                     // dist_sq != 0 (loss.py:15)
    const float r = d2 + softening, ir = 1.f / r, ir2 = ir * ir, ir4 = ir2 * ir2;
    const float dEdR = 4.f * (-6.f * ir4 * ir2 * ir + 3.f * ir4);
    fx += dEdR * 2.f * dx;
    fy += dEdR * 2.f * dy;
    fz += dEdR * 2.f * dz;
  }
  fx = wave_sum(fx);
  fy = wave_sum(fy);
  fz = wave_sum(fz);
  if (lane == 0) {
    apos[(size_t)a * 3 + 0] = cH * fx;
    apos[(size_t)a * 3 + 1] = cH * fy;
    apos[(size_t)a * 3 + 2] = cH * fz;
  }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static inline hipStream_t SB(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline int hid_ok_b(int H) { return H == 32 || H == 64 || H == 128; }
static inline size_t al64(size_t x) { return (x + 63) & ~(size_t)63; }
static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// Workspace: the per-layer pair-row / atom-row / partial sections come in
// BWD_NBUF copies (`span` floats apart): layer l's weight-gradient pass (outer
// kernels, on an auxiliary stream) reads buffer l % BWD_NBUF while the layer
// backwards of l-1, l-2 write the others.  Three buffers let the layer chain
// run two layers ahead of the weight-gradient passes instead of waiting on
// each one (backward -2.7 %, profiles/r02/r02y_ab_nbuf.txt; +6.6 GB at the
// bench batch); the large-system path and single layers use two.
#ifndef BWD_NBUF
#define BWD_NBUF 3
#endif
static_assert(BWD_NBUF >= 2, "at least double buffered");
struct BwdWs {
  size_t offs, buf0, span;   // shared offsets section; first buffer; buffer stride
  // offsets within a buffer (floats)
  size_t xin, p0, pe, pc, dp0, dpe, aphi, patt, dlogit, tmax, su, au, sn, an, aq, agr, anet, part, total;
  int nbuf;                  // buffers rotated by the layer chain (BWD_NBUF or 2)
  size_t part_floats;
};

static BwdWs bwd_ws(int num_mols, int num_atoms, int nf, int H, int n_layers, long long prb, int nbuf_cap = BWD_NBUF) {
  BwdWs W;
  size_t o = 0;
  const size_t P = (size_t)prb, A = (size_t)num_atoms;
  W.offs = 0;
  W.buf0 = al64((size_t)n_layers * (num_mols + 1));
  W.xin = o; o += al64(P * xin_width(nf));
  W.p0 = W.pc = 0;   // not stored (recomputed, see BwdArgs)
  W.pe = o; o += al64(P * H);
  W.dp0 = o; o += al64(P * H);
  W.dpe = o; o += al64(P * H);
  W.aphi = o; o += al64(P);
  W.patt = o; o += al64(P);
  W.dlogit = o; o += al64(P);
  W.tmax = o; o += al64((P / 32 + 1) * TMX_W);
  W.su = o; o += al64(A * H);
  W.au = o; o += al64(A * H);
  W.sn = o; o += al64(A * H);
  W.an = o; o += al64(A * H);
  W.aq = o; o += al64(A);
  W.agr = o; o += al64(A * nf);
  W.anet = o; o += al64(A * 2 * nf);
  const size_t chp = (size_t)cdiv(prb, OA_CHUNK), cha = (size_t)cdiv(num_atoms, OA_CHUNK_ATOM);
  // partials of one layer's 8 gradients (all in flight together)
  W.part_floats = chp * ((size_t)H * (2 * nf + 2) + 2 * (size_t)H * (H + 1) + H + (H + 1)) +   // + att_nn
                  cha * ((size_t)H * (nf + 1) + (H + 1) + (size_t)H * (H + nf + 1) + (size_t)nf * (H + 1));
  const size_t am = cha * ((size_t)H * (nf + 1) + (size_t)2 * nf * (H + 1));
  if (am > W.part_floats) W.part_floats = am;
  W.part = o; o += al64(W.part_floats);
  W.span = o;
  // fused layer chains of >= BWD_NBUF layers rotate BWD_NBUF buffers; the
  // large-system path (n_layers 0 here) and single-layer callers use two
  W.nbuf = n_layers >= nbuf_cap ? nbuf_cap : 2;
  W.total = W.buf0 + (size_t)W.nbuf * W.span;
  return W;
}

// Auxiliary stream (per device) for the weight-gradient passes, and a pool of
// sync events.  Host-side state only; guarded by a mutex (one backward's launch
// sequence at a time per process).
#include <mutex>
#include <stdlib.h>
#include <vector>
namespace {
struct AuxDev {
  hipStream_t s = nullptr;
  std::vector<hipEvent_t> ev;
};
std::mutex g_aux_mu;
AuxDev g_aux[64];
#ifdef ENFLOW_CHAIN_PRIO
// A/B: the layer chain on a high-priority stream of its own (the weight-gradient
// passes on the default-priority aux stream fill the CUs it leaves)
hipStream_t chain_stream(int dev) {
  static hipStream_t s[64] = {};
  if (!s[dev]) {
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (hipStreamCreateWithPriority(&s[dev], hipStreamNonBlocking, hi) != hipSuccess) s[dev] = nullptr;
  }
  return s[dev];
}
#endif
hipStream_t aux_stream(int dev) {
  if (!g_aux[dev].s) {   // created on `dev` (the caller's stream's device)
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
#ifdef ENFLOW_AUX_PRIO
    // A/B: the weight-gradient passes at another stream priority than the
    // layer chain (ENFLOW_AUX_PRIO = -1 / +1: lower / higher number = ...)
    {
      int lo = 0, hi = 0;
      hipDeviceGetStreamPriorityRange(&lo, &hi);
      const int pr = ENFLOW_AUX_PRIO > 0 ? hi : lo;
      if (hipStreamCreateWithPriority(&g_aux[dev].s, hipStreamNonBlocking, pr) != hipSuccess) g_aux[dev].s = nullptr;
    }
#else
    if (hipStreamCreateWithFlags(&g_aux[dev].s, hipStreamNonBlocking) != hipSuccess) g_aux[dev].s = nullptr;
#endif
    if (cur != dev) (void)hipSetDevice(cur);
  }
  return g_aux[dev].s;
}
hipEvent_t aux_event(int dev, size_t i) {
  auto& v = g_aux[dev].ev;
  while (v.size() <= i) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    v.push_back(e);
  }
  return v[i];
}
}  // namespace

static void add_desc(OuterBatch& ob, int& wg, const float* DY, int ldd, int M, const float* X, int ldx, int N,
                     const int32_t* rows_dev, int rows_static, int rows_bound, float*& part, float* outW,
                     float* outB, int tiled = 0) {
  OuterDesc& D = ob.d[ob.nd];
  D.tiled = tiled;
  D.xf_x = 0;
  D.xrow = nullptr;
  D.xf_dy = 0;
  D.rowv = nullptr;
  D.colv = nullptr;
  D.part2 = nullptr;
  D.recomp = RECOMP_NONE;
  D.Lp = nullptr;
  D.nf = 0;
  D.actp = nullptr;
  D.f32r = 0;
  D.tmaxA = D.tmaxB = nullptr;
  D.chunk = tiled ? OA_CHUNK : OA_CHUNK_ATOM;
  D.DY = DY; D.ldd = ldd; D.M = M; D.X = X; D.ldx = ldx; D.N = N;
  D.rows_dev = rows_dev; D.rows_static = rows_static;
  D.outW = outW; D.outB = outB;
  const int NB = N + (outB ? 1 : 0);
  D.mb = 1;
  D.nb = cdiv(N, 128);
  (void)NB;
  D.nch = rows_bound > 0 ? cdiv(rows_bound, D.chunk) : 0;
  D.part = part;
  part += (size_t)D.nch * M * NB;
  ob.start[ob.nd] = wg;
  wg += D.nch * D.nb;
  ++ob.nd;
  ob.start[ob.nd] = wg;
}

static int run_outer(OuterBatch& ob, int wg, hipStream_t st) {
  // one launch per layout (tile-blocked pair rows / row-major atom rows)
  for (int tl = 0; tl < 2; ++tl) {
    OuterBatch sub;
    sub.nd = 0;
    int swg = 0;
    for (int k = 0; k < ob.nd; ++k) {
      if (ob.d[k].tiled != tl) continue;
      sub.d[sub.nd] = ob.d[k];
      sub.start[sub.nd] = swg;
      swg += ob.start[k + 1] - ob.start[k];
      sub.start[++sub.nd] = swg;
    }
    if (swg > 0) {
      bool gen = false;   // a non-SiLU act_fn in the batch: the generic-activation instance
      for (int k = 0; k < sub.nd; ++k) gen |= sub.d[k].actp != nullptr;
      if (tl && gen) ENFLOW_TIMED("outer_acc_kernel", st, hipLaunchKernelGGL((outer_acc_kernel<true, true>), dim3(swg), dim3(256), 0, st, sub));
      else if (tl) ENFLOW_TIMED("outer_acc_kernel", st, hipLaunchKernelGGL((outer_acc_kernel<true, false>), dim3(swg), dim3(256), 0, st, sub));
      else ENFLOW_TIMED("outer_acc_kernel", st, hipLaunchKernelGGL((outer_acc_kernel<false, false>), dim3(swg), dim3(256), 0, st, sub));
    }
  }
  // F16X3 MFMA: tile-blocked descriptors with M > 1
  {
    OuterBatch sub;
    sub.nd = 0;
    int swg = 0;
    for (int k = 0; k < ob.nd; ++k) {
      if (ob.d[k].tiled != 2) continue;
      sub.d[sub.nd] = ob.d[k];
      sub.start[sub.nd] = swg;
      swg += ob.start[k + 1] - ob.start[k];
      sub.start[++sub.nd] = swg;
    }
    bool gen = false, f32r = false;
    for (int k = 0; k < sub.nd; ++k) {
      gen |= sub.d[k].actp != nullptr;
      f32r |= sub.d[k].f32r != 0;
    }
    if (swg > 0 && f32r) ENFLOW_TIMED("outer_x3_kernel", st, hipLaunchKernelGGL((outer_x3_kernel<true, true>), dim3(swg), dim3(256), 0, st, sub));
    else if (swg > 0 && gen) ENFLOW_TIMED("outer_x3_kernel", st, hipLaunchKernelGGL(outer_x3_kernel<true>, dim3(swg), dim3(256), 0, st, sub));
    else if (swg > 0) ENFLOW_TIMED("outer_x3_kernel", st, hipLaunchKernelGGL(outer_x3_kernel<false>, dim3(swg), dim3(256), 0, st, sub));
  }
  (void)wg;
  // reducer: one workgroup per 256 outputs of each descriptor
  OuterBatch rb = ob;
  int rw = 0;
  for (int k = 0; k < ob.nd; ++k) {
    rb.start[k] = rw;
    const int NB = ob.d[k].N + (ob.d[k].outB ? 1 : 0);
    rw += cdiv((long long)ob.d[k].M * NB, RP_OUT);
  }
  rb.start[ob.nd] = rw;
  if (rw > 0) ENFLOW_TIMED("reduce_part_kernel", st, hipLaunchKernelGGL(reduce_part_kernel, dim3(rw), dim3(256), 0, st, rb));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

#define DISPATCH_HN_B(H, NMAXSEL, CALL)                      \
  do {                                                        \
    if (NMAXSEL <= 32) {                                      \
      if (H == 32) { CALL(32, 32); }                          \
      else if (H == 64) { CALL(64, 32); }                     \
      else { CALL(128, 32); }                                 \
    } else {                                                  \
      if (H == 32) { CALL(32, 64); }                          \
      else if (H == 64) { CALL(64, 64); }                     \
      else { CALL(128, 64); }                                 \
    }                                                         \
  } while (0)

// One layer's weight gradients from its pair rows (prow: device count of pair
// rows) and atom rows, straight into the torch parameter layout G.
static int layer_weight_grads(hipStream_t st2, const BwdWs& Wl, float* wb, const int32_t* prow, int prb,
                              bool variants, float* G, const float* Rp, const RawEgcl& R, const float* hx,
                              int num_atoms, int nf, int H, const float* Lp, bool f32b = false) {
    OuterBatch ob;
    ob.nd = 0;
    int wg = 0;
    float* part = wb + Wl.part;
    const int XW = xin_width(nf);
    add_desc(ob, wg, wb + Wl.dp0, H, H, wb + Wl.xin, XW, 2 * nf + 1, prow, 0, prb, part, G + R.We1, G + R.be1,
             PAIR_OUTER);
    ob.d[ob.nd - 1].tmaxA = wb + Wl.tmax + TMX_DP0;
    ob.d[ob.nd - 1].tmaxB = wb + Wl.tmax + TMX_XIN;
    // edge_nn.2: X = silu(pre0), pre0 recomputed from the xin rows
    // the layer's act_fn (variant layers; packed layer + vfl + 1): the recomputed
    // activations and their derivatives follow it (NULL: SiLU instances)
    // (the fp32 backward always runs the generic instances)
    const float* actp = (variants || f32b) ? Lp + egcl_layout(H, nf).vfl + 1 : nullptr;
    add_desc(ob, wg, wb + Wl.dpe, H, H, wb + Wl.xin, XW, H, prow, 0, prb, part, G + R.We2, G + R.be2, PAIR_OUTER);
    ob.d[ob.nd - 1].recomp = RECOMP_X0;
    ob.d[ob.nd - 1].tmaxA = wb + Wl.tmax + TMX_DPE;
    ob.d[ob.nd - 1].tmaxB = wb + Wl.tmax + TMX_X1;
    ob.d[ob.nd - 1].Lp = Lp;
    ob.d[ob.nd - 1].nf = nf;
    ob.d[ob.nd - 1].actp = actp;
    ob.d[ob.nd - 1].f32r = f32b;
    // coord_nn.0: X = silu(pre_e) = the message; DY = aphi * wc2 * silu'(pc), pc recomputed from X
    add_desc(ob, wg, nullptr, H, H, wb + Wl.pe, H, H, prow, 0, prb, part,
             G + R.Wc1, G + R.bc1, PAIR_OUTER);
    ob.d[ob.nd - 1].xf_x = 1;
    ob.d[ob.nd - 1].xf_dy = 1;
    ob.d[ob.nd - 1].rowv = wb + Wl.aphi;
    if (variants) ob.d[ob.nd - 1].xrow = wb + Wl.patt;          // the message is e * att
    ob.d[ob.nd - 1].colv = Rp + R.wc2;
    ob.d[ob.nd - 1].recomp = RECOMP_PC;
    ob.d[ob.nd - 1].tmaxA = wb + Wl.tmax + TMX_DPC;
    ob.d[ob.nd - 1].tmaxB = wb + Wl.tmax + TMX_MSG;
    ob.d[ob.nd - 1].Lp = Lp;
    ob.d[ob.nd - 1].nf = nf;
    ob.d[ob.nd - 1].actp = actp;
    ob.d[ob.nd - 1].f32r = f32b;
    // coord_nn.2: d wc2 = sum_rows aphi silu(pc), folded into coord_nn.0's pass (its partials
    // written there; this descriptor only sizes them and feeds the reduction)
    add_desc(ob, wg, wb + Wl.aphi, 1, 1, nullptr, H, H, prow, 0, prb, part, G + R.wc2, nullptr, 3);
    ob.d[ob.nd - 2].part2 = ob.d[ob.nd - 1].part;
    if (variants) {   // att_nn.0: d w = sum_rows dlogit e, d b = sum_rows dlogit (0 rows without attention)
      add_desc(ob, wg, wb + Wl.dlogit, 1, 1, wb + Wl.pe, H, H, prow, 0, prb, part, G + R.watt, G + R.batt, 1);
      ob.d[ob.nd - 1].xf_x = 1;                                 // X = silu(pre_e) = e
      ob.d[ob.nd - 1].actp = actp;
    }
    add_desc(ob, wg, wb + Wl.au, H, H, hx, nf + H, nf, nullptr, num_atoms, num_atoms, part, G + R.Wv1, G + R.bv1);
    add_desc(ob, wg, wb + Wl.aq, 1, 1, wb + Wl.su, H, H, nullptr, num_atoms, num_atoms, part, G + R.Wv2, G + R.bv2);
    add_desc(ob, wg, wb + Wl.an, H, H, hx, nf + H, nf + H, nullptr, num_atoms, num_atoms, part, G + R.Wn1,
             G + R.bn1);
    add_desc(ob, wg, wb + Wl.agr, nf, nf, wb + Wl.sn, H, H, nullptr, num_atoms, num_atoms, part, G + R.Wn2,
             G + R.bn2);
    return run_outer(ob, wg, st2);
}

// ArgMax.network's gradients (the flow's dequantiser) into grad_dequant; ptr /
// chunks: the atom chunks argmax_bwd_kernel runs on (<= nmax_sel atoms each)
static int argmax_grads(hipStream_t st, const BwdWs& Wl, float* wb, const int32_t* ptr, int chunks, int nmax_sel,
                        int H, int nf, int num_atoms, const float* h_data, const float* noise,
                        const float* dequant_raw, const float* adj_h, const float* adj_ldj, float* grad_dequant) {
    float* apre = wb + Wl.au;
    float* spre = wb + Wl.su;
    float* anet = wb + Wl.anet;
#define CALL(HH, NN)                                                                                    \
  hipLaunchKernelGGL((argmax_bwd_kernel<HH, NN>), dim3(chunks), dim3(BLOCK), 0, st, ptr, nf, h_data, noise, \
                     dequant_raw, adj_h, adj_ldj, apre, spre, anet)
    DISPATCH_HN_B(H, nmax_sel, CALL);
#undef CALL
    const int rW1 = 0, rb1 = H * nf, rW2 = rb1 + H, rb2 = rW2 + 2 * nf * H;
    OuterBatch ob;
    ob.nd = 0;
    int wg = 0;
    float* part = wb + Wl.part;
    add_desc(ob, wg, apre, H, H, h_data, nf, nf, nullptr, num_atoms, num_atoms, part, grad_dequant + rW1,
             grad_dequant + rb1);
    add_desc(ob, wg, anet, 2 * nf, 2 * nf, spre, H, H, nullptr, num_atoms, num_atoms, part, grad_dequant + rW2,
             grad_dequant + rb2);
    return run_outer(ob, wg, st);
}

extern "C" {

#if defined(ENFLOW_STAMPS_BWD) && !defined(ENFLOW_STAMPS)
int enflow_read_stamps(unsigned long long* host_out, int reset) {
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(enflow_stamp_acc), sizeof(unsigned long long) * NSTAMP) != hipSuccess)
    return -2;
  if (reset) {
    unsigned long long z[NSTAMP] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(enflow_stamp_acc), z, sizeof(z)) != hipSuccess) return -2;
  }
  return NSTAMP;
}
#endif

int64_t enflow_lf_tape_size(int num_atoms, int nf, int H, int n_layers) {
  if (num_atoms < 0 || nf < 1 || nf > BWD_NFMAX || !hid_ok_b(H) || n_layers < 0) return -1;
  return (int64_t)tape_layout(num_atoms, nf, H, n_layers).total;
}

// The neighbour-list section (pair words and row counts, the layout's tail) is
// written by the 33..64-atom fused forward and read back by its backward only;
// other batches' tapes end before it.
int64_t enflow_lf_tape_size_for(int num_atoms, int nf, int H, int n_layers, int max_mol_atoms) {
  if (num_atoms < 0 || nf < 1 || nf > BWD_NFMAX || !hid_ok_b(H) || n_layers < 0 || max_mol_atoms < 0) return -1;
  const TapeLayout T = tape_layout(num_atoms, nf, H, n_layers);
  static_assert(TAPE_PAIR_CAP + 1 == 64, "the pair section belongs to the 64-atom instance");
  return (int64_t)(max_mol_atoms > 32 && max_mol_atoms <= TAPE_PAIR_CAP + 1 ? T.total : T.pairs);
}

int64_t enflow_egcl_bwd_packed_size(int H, int nf) {
  if (!hid_ok_b(H) || nf < 1 || nf > BWD_NFMAX) return -1;
  return egcl_bwd_layout(H).total;
}

int enflow_pack_egcl_bwd_f32(const float* raw, int H, int nf, float* packed, void* stream) {
  if (!hid_ok_b(H) || nf < 1 || nf > BWD_NFMAX || !raw || !packed) return -1;
  const int total = egcl_bwd_layout(H).total;
  hipLaunchKernelGGL(egcl_bwd_scale_kernel, dim3(6), dim3(256), 0, SB(stream), raw, H, nf, packed);
  hipLaunchKernelGGL(pack_egcl_bwd_kernel, dim3(cdiv(total, 256)), dim3(256), 0, SB(stream), raw, H, nf, packed);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int enflow_pack_egcl_bwd_layers_f32(const float* raw, int64_t raw_stride, int n_layers, int H, int nf,
                                    float* packed, void* stream) {
  if (!hid_ok_b(H) || nf < 1 || nf > BWD_NFMAX || !raw || !packed || n_layers < 0 || n_layers > 65535) return -1;
  if (raw_stride < raw_egcl(H, nf).total) return -1;
  if (n_layers == 0) return 0;
  const int total = egcl_bwd_layout(H).total;
  hipLaunchKernelGGL(egcl_bwd_scale_layers_kernel, dim3(6, n_layers), dim3(256), 0, SB(stream), raw, raw_stride, H, nf,
                     packed, (int64_t)total);
  hipLaunchKernelGGL(pack_egcl_bwd_layers_kernel, dim3(cdiv(total, 256), n_layers), dim3(256), 0, SB(stream), raw,
                     raw_stride, H, nf, packed, (int64_t)total);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int64_t enflow_lf_backward_workspace_size(int num_mols, int num_atoms, int nf, int H, int n_layers,
                                          int64_t pair_row_bound) {
  if (num_mols < 0 || num_atoms < 0 || nf < 1 || nf > BWD_NFMAX || !hid_ok_b(H) || n_layers < 0 || pair_row_bound < 0)
    return -1;
  return (int64_t)(bwd_ws(num_mols, num_atoms, nf, H, n_layers, pair_row_bound).total * sizeof(float));
}

int64_t enflow_lf_backward_workspace_size_min(int num_mols, int num_atoms, int nf, int H, int n_layers,
                                              int64_t pair_row_bound) {
  if (num_mols < 0 || num_atoms < 0 || nf < 1 || nf > BWD_NFMAX || !hid_ok_b(H) || n_layers < 0 || pair_row_bound < 0)
    return -1;
  return (int64_t)(bwd_ws(num_mols, num_atoms, nf, H, n_layers, pair_row_bound, 2).total * sizeof(float));
}

int enflow_alchemical_nll_backward_f32(int num_mols, int num_atoms, int max_mol_atoms, int nf,
                                       const int32_t* mol_ptr, const float* h, const float* g,
                                       const float* pos, const float* vel, float kBT, float softening,
                                       const float* grad_loss, float* adj_h, float* adj_g, float* adj_pos,
                                       float* adj_vel, float* adj_ldj, void* stream) {
  if (num_mols < 1 || num_atoms < 0 || nf < 1 || !adj_ldj) return -1;
  const int tm = enflow_tm_begin("nll_bwd_kernel", SB(stream));
  if (max_mol_atoms > 64)
    hipLaunchKernelGGL(nll_bwd_large_kernel, dim3(num_atoms / WAVES + 1), dim3(BLOCK), 0, SB(stream), mol_ptr,
                       num_mols, num_atoms, nf, h, g, pos, vel, kBT, softening, grad_loss, adj_h, adj_g, adj_pos,
                       adj_vel, adj_ldj);
  else if (max_mol_atoms <= 32)
    hipLaunchKernelGGL((nll_bwd_kernel<32>), dim3(num_mols), dim3(BLOCK), 0, SB(stream), mol_ptr, num_mols, nf, h, g,
                       pos, vel, kBT, softening, grad_loss, adj_h, adj_g, adj_pos, adj_vel, adj_ldj);
  else
    hipLaunchKernelGGL((nll_bwd_kernel<64>), dim3(num_mols), dim3(BLOCK), 0, SB(stream), mol_ptr, num_mols, nf, h, g,
                       pos, vel, kBT, softening, grad_loss, adj_h, adj_g, adj_pos, adj_vel, adj_ldj);
  enflow_tm_end(tm, SB(stream));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

static int lf_backward_impl(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                            const int32_t* mol_ptr, const float* r_cut, const float* box,
                            const float* tape, const int32_t* pair_counts,
                            const float* layers, const float* layers_bwd, const float* layers_raw, int n_layers,
                            int dequant_kind, const float* dequant_raw, const float* h_data, const float* noise,
                            float dt, float cw,
                            float* adj_h, float* adj_g, float* adj_pos, float* adj_vel, const float* adj_ldj,
                            float* grad_layers, float* grad_dequant,
                            void* workspace, int64_t workspace_bytes, int64_t pair_row_bound,
                            int32_t* err_flag, void* stream,
                            const float* eg_dQ, const float* eg_dF, const float* eg_dG) {
  // dequant_kind may carry ENFLOW_EGCL_VARIANTS (layers with norm_diff / tanh
  // flags) and ENFLOW_BWD_F32 (the tape of an fp32-GEMM forward: fp32 backward)
  const bool variants = (dequant_kind & ENFLOW_EGCL_VARIANTS) != 0;
  const bool f32b = (dequant_kind & ENFLOW_BWD_F32) != 0;
  dequant_kind &= 0xff;
  if (num_mols < 0 || num_atoms < 0 || max_mol_atoms < 0 || max_mol_atoms > 64 || nf < 1 || nf > BWD_NFMAX ||
      !hid_ok_b(H) || n_layers < 0 || pair_row_bound < 0 || pair_row_bound > 0x7fffffffLL)
    return -1;
  if (!tape || !pair_counts || !layers || !layers_bwd || !layers_raw || !adj_h || !adj_g || !adj_pos ||
      !adj_vel || !adj_ldj || !grad_layers || !workspace || !err_flag)
    return -1;
  if (dequant_kind == ENFLOW_DEQUANT_ARGMAX && (!dequant_raw || !h_data || !noise || !grad_dequant)) return -1;
  // BWD_NBUF rotating buffers when the workspace holds them, else two (the
  // layer chain then waits for the weight-gradient pass two layers up)
  BwdWs Wl = bwd_ws(num_mols, num_atoms, nf, H, n_layers, pair_row_bound);
  if ((uint64_t)workspace_bytes < Wl.total * sizeof(float)) Wl = bwd_ws(num_mols, num_atoms, nf, H, n_layers, pair_row_bound, 2);
  if ((uint64_t)workspace_bytes < Wl.total * sizeof(float)) return -6;
  if (num_mols == 0) return 0;
  hipStream_t st = SB(stream);
  float* ws = reinterpret_cast<float*>(workspace);
  int32_t* offs = reinterpret_cast<int32_t*>(ws + Wl.offs);
  const EgclLayout L = egcl_layout(H, nf);
  const EgclBwdLayout LB = egcl_bwd_layout(H);
  const RawEgcl R = raw_egcl(H, nf);
  const int prb = (int)pair_row_bound;
  // weight-gradient passes of layer l run on an auxiliary stream, overlapping the
  // layer backward of l - 1 (double-buffered rows); the caller's stream joins it
  // before the dequantiser's gradients and before returning
  int dev = 0;
  if ((st ? hipStreamGetDevice(st, &dev) : hipGetDevice(&dev)) != hipSuccess || dev < 0 || dev >= 64) return -2;
  std::lock_guard<std::mutex> aux_lock(g_aux_mu);
  const bool serial = getenv("ENFLOW_SERIAL_BWD") != nullptr;   // diagnostic: no overlap
  hipStream_t st2 = aux_stream(dev);
  if (!st2) return -2;
  auto ev = [&](int i) { return aux_event(dev, (size_t)i); };   // 2 l: backward of l done, 2 l + 1: outer of l done
  for (int i = 0; i < 2 * n_layers + 1; ++i)
    if (!ev(i)) return -2;

  hipStream_t st_caller = st;
#ifdef ENFLOW_CHAIN_PRIO
  hipStream_t sth = chain_stream(dev);
  if (!sth || !ev(2 * n_layers)) return -2;
  if (hipEventRecord(ev(2 * n_layers), st) != hipSuccess || hipStreamWaitEvent(sth, ev(2 * n_layers), 0) != hipSuccess)
    return -2;
  st = sth;
#endif
  if (n_layers > 0)
    hipLaunchKernelGGL(pair_offsets_kernel, dim3(n_layers), dim3(BLOCK), 0, st, pair_counts, num_mols, offs);

  for (int l = n_layers - 1; l >= 0; --l) {
    float* const wb = ws + Wl.buf0 + (size_t)(l % Wl.nbuf) * Wl.span;   // this layer's buffer
    // the buffer was last read by layer l + nbuf's weight-gradient pass
    if (l + Wl.nbuf < n_layers && hipStreamWaitEvent(st, ev(2 * (l + Wl.nbuf) + 1), 0) != hipSuccess)
      return -2;
    BwdArgs A{};
    A.mol_ptr = mol_ptr; A.r_cut = r_cut; A.box = box; A.tape = tape;
    A.num_atoms = num_atoms; A.num_mols = num_mols; A.n_layers = n_layers; A.layer = l; A.nf = nf;
    A.Lp = layers + (size_t)l * L.total;
    A.Bp = layers_bwd + (size_t)l * LB.total;
    A.Rp = layers_raw + (size_t)l * R.total_bwd;
    A.dt = dt; A.cw = cw; A.adj_ldj = adj_ldj;
    A.ah = adj_h; A.ag = adj_g; A.apos = adj_pos; A.avel = adj_vel;
    A.pair_off = offs + (size_t)l * (num_mols + 1);
    A.xin = wb + Wl.xin; A.p0 = nullptr; A.pe = wb + Wl.pe; A.pc = nullptr;
    A.dp0 = wb + Wl.dp0; A.dpe = wb + Wl.dpe; A.aphi = wb + Wl.aphi;
    A.patt = wb + Wl.patt; A.dlogit = wb + Wl.dlogit; A.tmax = wb + Wl.tmax;
    A.su = wb + Wl.su; A.au = wb + Wl.au; A.sn = wb + Wl.sn; A.an = wb + Wl.an;
    A.aq = wb + Wl.aq; A.agr = wb + Wl.agr; A.err = err_flag;
    A.eg_dQ = eg_dQ; A.eg_dF = eg_dF; A.eg_dG = eg_dG;
    A.pair_counts_l = pair_counts + (size_t)l * num_mols;
    // the forward's 64-atom instance tapes the list (molecules of 33..64 atoms; see flow_kernel.h)
    A.tape_pairs = eg_dQ == nullptr && max_mol_atoms > 32 && !getenv("ENFLOW_BWD_REBUILD_PAIRS");
    if (f32b) {   // generic (VAR) instance: any flags / act_fn
#define CALL(HH, NN) ENFLOW_TIMED("lf_layer_bwd_kernel", st, hipLaunchKernelGGL((lf_layer_bwd_kernel<HH, NN, true, PREC_F32>), dim3(num_mols), dim3(BLOCK), 0, st, A))
      DISPATCH_HN_B(H, max_mol_atoms, CALL);
#undef CALL
    } else if (variants) {
#define CALL(HH, NN) ENFLOW_TIMED("lf_layer_bwd_kernel", st, hipLaunchKernelGGL((lf_layer_bwd_kernel<HH, NN, true>), dim3(num_mols), dim3(BLOCK), 0, st, A))
      DISPATCH_HN_B(H, max_mol_atoms, CALL);
#undef CALL
    } else {
#define CALL(HH, NN) ENFLOW_TIMED("lf_layer_bwd_kernel", st, hipLaunchKernelGGL((lf_layer_bwd_kernel<HH, NN, false>), dim3(num_mols), dim3(BLOCK), 0, st, A))
      DISPATCH_HN_B(H, max_mol_atoms, CALL);
#undef CALL
    }
    if (hipEventRecord(ev(2 * l), st) != hipSuccess || hipStreamWaitEvent(st2, ev(2 * l), 0) != hipSuccess)
      return -2;
    // the layer's weight gradients, straight into the torch parameter layout (aux stream)
    const int rc = layer_weight_grads(st2, Wl, wb, offs + (size_t)l * (num_mols + 1) + num_mols, prb, variants,
                                      grad_layers + (size_t)l * R.total_bwd, A.Rp, R,
                                      tape + tape_layout(num_atoms, nf, H, n_layers).hx +
                                          (size_t)l * num_atoms * (nf + H),
                                      num_atoms, nf, H, A.Lp, f32b);
    if (rc) return rc;
    if (hipEventRecord(ev(2 * l + 1), st2) != hipSuccess) return -2;
    if (serial && hipStreamWaitEvent(st, ev(2 * l + 1), 0) != hipSuccess) return -2;
  }
#ifdef ENFLOW_CHAIN_PRIO
  if (hipEventRecord(ev(2 * n_layers), st) != hipSuccess || hipStreamWaitEvent(st_caller, ev(2 * n_layers), 0) != hipSuccess)
    return -2;
#endif
  st = st_caller;
  // join: every weight-gradient pass done before the dequantiser's (buffer 0 again) and the return
  if (n_layers > 0 && hipStreamWaitEvent(st, ev(1), 0) != hipSuccess) return -2;   // layer 0's pass (the last)

  if (dequant_kind == ENFLOW_DEQUANT_ARGMAX) {
    const int rc = argmax_grads(st, Wl, ws + Wl.buf0, mol_ptr, num_mols, max_mol_atoms, H, nf, num_atoms, h_data,
                                noise, dequant_raw, adj_h, adj_ldj, grad_dequant);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(poison_on_err_kernel, dim3(64), dim3(256), 0, st, err_flag, grad_layers,
                     (long long)n_layers * R.total_bwd, dequant_kind == ENFLOW_DEQUANT_ARGMAX ? grad_dequant : nullptr,
                     (long long)(H * nf + H + 2 * nf * H + 2 * nf));   // ArgMax.network: W1, b1, W2, b2
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int enflow_lf_backward_f32(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                           const int32_t* mol_ptr, const float* r_cut, const float* box,
                           const float* tape, const int32_t* pair_counts,
                           const float* layers, const float* layers_bwd, const float* layers_raw, int n_layers,
                           int dequant_kind, const float* dequant_raw, const float* h_data, const float* noise,
                           float dt, float cw,
                           float* adj_h, float* adj_g, float* adj_pos, float* adj_vel, const float* adj_ldj,
                           float* grad_layers, float* grad_dequant,
                           void* workspace, int64_t workspace_bytes, int64_t pair_row_bound,
                           int32_t* err_flag, void* stream) {
  return lf_backward_impl(num_mols, num_atoms, max_mol_atoms, nf, H, mol_ptr, r_cut, box, tape, pair_counts, layers,
                          layers_bwd, layers_raw, n_layers, dequant_kind, dequant_raw, h_data, noise, dt, cw, adj_h,
                          adj_g, adj_pos, adj_vel, adj_ldj, grad_layers, grad_dequant, workspace, workspace_bytes,
                          pair_row_bound, err_flag, stream, nullptr, nullptr, nullptr);
}

// ---- large systems (molecules past the fused backward's 64-atom image) -----
// Per layer, last to first: the neighbour list of the layer's taped positions
// (the forward's own search kernels, + the dense slot map), the pair-row offsets
// of the row blocks, lf_layer_bwd_kernel<.., BIG> per block of rows (row-side
// adjoints in LDS, column-side per pair into colc), the column sums (colsum per
// row chunk, colfinal per id_mapping label), then the weight gradients on the
// auxiliary stream as in the fused backward.
struct LgBwdWs { size_t lg, smap, bwd, colc, part, boff, tot, rowstart, chunk, total; int nch, nb; };
static LgBwdWs lg_bwd_ws(int num_mols, int num_atoms, int max_n, int nf, int H, long long prb) {
  LgBwdWs W;
  const size_t A = (size_t)num_atoms;
  W.nch = max(1, cdiv(max_n, LG_RC));
  W.nb = num_atoms / lg_rows(num_atoms) + num_mols + 1;
  size_t o = 0;
  W.lg = o; o = al256(o + lg_workspace(num_mols, num_atoms, max_n, nf).total);
  W.smap = o; o = al256(o + A * (size_t)max_n * 4);
  W.bwd = o; o = al256(o + bwd_ws(num_mols, num_atoms, nf, H, 0, prb).total * sizeof(float));
  W.colc = o; o = al256(o + (size_t)prb * CSTR * 4);
  W.part = o; o = al256(o + (size_t)W.nch * A * CSTR * 4);
  W.boff = o; o = al256(o + 2 * ((size_t)W.nb + 1) * 4);
  W.tot = o; o = al256(o + 2 * 4);
  W.rowstart = o; o = al256(o + A * 4);
  W.chunk = o; o = al256(o + ((A + 31) / 32 + 2) * 4);
  W.total = o;
  return W;
}

int64_t enflow_lf_backward_large_workspace_size(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                                                int64_t pair_row_bound) {
  if (num_mols < 0 || num_atoms < 0 || max_mol_atoms < 0 || max_mol_atoms >= (1 << 22) || nf < 1 || nf > BWD_NFMAX ||
      !hid_ok_b(H) || pair_row_bound < 0 || pair_row_bound > 0x7fffffffLL)
    return -1;
  return (int64_t)lg_bwd_ws(num_mols, num_atoms, max_mol_atoms, nf, H, pair_row_bound).total;
}

static int lf_backward_large_impl(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                                  const int32_t* mol_ptr, const float* r_cut, const float* box, const float* tape,
                                  const float* layers, const float* layers_bwd, const float* layers_raw,
                                  int n_layers, int dequant_kind, const float* dequant_raw, const float* h_data,
                                  const float* noise, float dt, float cw, float* adj_h, float* adj_g,
                                  float* adj_pos, float* adj_vel, const float* adj_ldj, float* grad_layers,
                                  float* grad_dequant, void* workspace, int64_t workspace_bytes,
                                  int64_t pair_row_bound, int32_t* err_flag, void* stream, const float* eg_dQ,
                                  const float* eg_dF, const float* eg_dG) {
  const bool variants = (dequant_kind & ENFLOW_EGCL_VARIANTS) != 0;
  const bool f32b = (dequant_kind & ENFLOW_BWD_F32) != 0;
  dequant_kind &= 0xff;
  const int64_t need = enflow_lf_backward_large_workspace_size(num_mols, num_atoms, max_mol_atoms, nf, H,
                                                               pair_row_bound);
  if (need < 0 || n_layers < 0) return -1;
  if (!mol_ptr || !r_cut || !box || !tape || !layers || !layers_bwd || !layers_raw || !adj_h || !adj_g ||
      !adj_pos || !adj_vel || !adj_ldj || !grad_layers || !workspace || !err_flag)
    return -1;
  if (dequant_kind == ENFLOW_DEQUANT_ARGMAX && (!dequant_raw || !h_data || !noise || !grad_dequant)) return -1;
  if (workspace_bytes < need) return -6;
  if (num_mols == 0) return 0;
  const LgBwdWs W = lg_bwd_ws(num_mols, num_atoms, max_mol_atoms, nf, H, pair_row_bound);
  const BwdWs Wl = bwd_ws(num_mols, num_atoms, nf, H, 0, pair_row_bound);
  char* base = static_cast<char*>(workspace);
  float* ws = reinterpret_cast<float*>(base + W.bwd);
  int32_t* smap = reinterpret_cast<int32_t*>(base + W.smap);
  float* colc = reinterpret_cast<float*>(base + W.colc);
  float* part = reinterpret_cast<float*>(base + W.part);
  int32_t* boff = reinterpret_cast<int32_t*>(base + W.boff);
  int32_t* tot = reinterpret_cast<int32_t*>(base + W.tot);
  int32_t* rowstart = reinterpret_cast<int32_t*>(base + W.rowstart);
  int32_t* chunk = reinterpret_cast<int32_t*>(base + W.chunk);
  hipStream_t st = SB(stream);
  const EgclLayout L = egcl_layout(H, nf);
  const EgclBwdLayout LB = egcl_bwd_layout(H);
  const RawEgcl R = raw_egcl(H, nf);
  const TapeLayout T = tape_layout(num_atoms, nf, H, n_layers);
  const int prb = (int)pair_row_bound;
  LgArgs G = lg_args(num_mols, num_atoms, max_mol_atoms, nf, mol_ptr, r_cut, box, nullptr, nullptr, nullptr,
                     nullptr, dt, cw, err_flag, base + W.lg);
  G.smap = smap;
  int dev = 0;
  if ((st ? hipStreamGetDevice(st, &dev) : hipGetDevice(&dev)) != hipSuccess || dev < 0 || dev >= 64) return -2;
  std::lock_guard<std::mutex> aux_lock(g_aux_mu);
  const bool serial = getenv("ENFLOW_SERIAL_BWD") != nullptr;   // diagnostic: no overlap
  hipStream_t st2 = aux_stream(dev);
  if (!st2) return -2;
  auto ev = [&](int i) { return aux_event(dev, (size_t)i); };
  for (int i = 0; i < 2 * n_layers + 1; ++i)
    if (!ev(i)) return -2;
  lg_setup(st, G);
  const int grid = lg_grid(G);
  const int ga = (num_atoms + BLOCK - 1) / BLOCK;
  for (int l = n_layers - 1; l >= 0; --l) {
    float* const wb = ws + Wl.buf0 + (size_t)(l & 1) * Wl.span;
    int32_t* const boff_l = boff + (size_t)(l & 1) * (W.nb + 1);
    int32_t* const tot_l = tot + (l & 1);
    if (l + 2 < n_layers && hipStreamWaitEvent(st, ev(2 * (l + 2) + 1), 0) != hipSuccess) return -2;
    G.pos = const_cast<float*>(tape + T.pos + (size_t)l * num_atoms * 3);
    lg_search(st, G);
    ENFLOW_TIMED("lg_bwd_offsets_kernel", st, hipLaunchKernelGGL(lg_bwd_offsets_kernel, dim3(1), dim3(BLOCK), 0, st, mol_ptr, num_mols, G.blk_start, G.rbl,
                       G.npairs, boff_l, tot_l));
    BwdArgs A{};
    A.mol_ptr = mol_ptr; A.r_cut = r_cut; A.box = box; A.tape = tape;
    A.num_atoms = num_atoms; A.num_mols = num_mols; A.n_layers = n_layers; A.layer = l; A.nf = nf;
    A.Lp = layers + (size_t)l * L.total;
    A.Bp = layers_bwd + (size_t)l * LB.total;
    A.Rp = layers_raw + (size_t)l * R.total_bwd;
    A.dt = dt; A.cw = cw; A.adj_ldj = adj_ldj;
    A.ah = adj_h; A.ag = adj_g; A.apos = adj_pos; A.avel = adj_vel;
    A.xin = wb + Wl.xin; A.p0 = nullptr; A.pe = wb + Wl.pe; A.pc = nullptr;
    A.dp0 = wb + Wl.dp0; A.dpe = wb + Wl.dpe; A.aphi = wb + Wl.aphi;
    A.patt = wb + Wl.patt; A.dlogit = wb + Wl.dlogit; A.tmax = wb + Wl.tmax;
    A.su = wb + Wl.su; A.au = wb + Wl.au; A.sn = wb + Wl.sn; A.an = wb + Wl.an;
    A.aq = wb + Wl.aq; A.agr = wb + Wl.agr; A.err = err_flag;
    A.blk_start = G.blk_start; A.rbl = G.rbl; A.max_n = max_mol_atoms;
    A.npairs_g = G.npairs; A.cntrow_g = G.cntrow; A.pairs_g = G.pairs;
    A.boff = boff_l; A.rowstart = rowstart; A.colc = colc; A.prb = pair_row_bound;
    A.eg_dQ = eg_dQ; A.eg_dF = eg_dF; A.eg_dG = eg_dG;
#define CALLB(HH)                                                                                              \
  do {                                                                                                         \
    if (f32b) ENFLOW_TIMED("lf_layer_bwd_kernel", st, hipLaunchKernelGGL((lf_layer_bwd_kernel<HH, 32, true, PREC_F32, true>), dim3(grid), dim3(BLOCK), 0, st, A)); \
    else if (variants) ENFLOW_TIMED("lf_layer_bwd_kernel", st, hipLaunchKernelGGL((lf_layer_bwd_kernel<HH, 32, true, ENFLOW_BWD_PREC, true>), dim3(grid), dim3(BLOCK), 0, st, A)); \
    else ENFLOW_TIMED("lf_layer_bwd_kernel", st, hipLaunchKernelGGL((lf_layer_bwd_kernel<HH, 32, false, ENFLOW_BWD_PREC, true>), dim3(grid), dim3(BLOCK), 0, st, A)); \
  } while (0)
    if (H == 32) CALLB(32);
    else if (H == 64) CALLB(64);
    else CALLB(128);
#undef CALLB
    if (num_atoms > 0) {
      ENFLOW_TIMED("lg_colsum_kernel", st, hipLaunchKernelGGL(lg_colsum_kernel, dim3(ga, W.nch), dim3(BLOCK), 0, st, mol_ptr, num_mols, num_atoms,
                         max_mol_atoms, smap, rowstart, colc, nf, part));
      ENFLOW_TIMED("lg_colfinal_kernel", st, hipLaunchKernelGGL(lg_colfinal_kernel, dim3((num_atoms + WAVES - 1) / WAVES), dim3(BLOCK), 0, st, mol_ptr, num_mols, num_atoms, G.idmap,
                         part, W.nch, nf, adj_h, adj_pos));
    }
    if (hipEventRecord(ev(2 * l), st) != hipSuccess || hipStreamWaitEvent(st2, ev(2 * l), 0) != hipSuccess)
      return -2;
    const int rc = layer_weight_grads(st2, Wl, wb, tot_l, prb, variants, grad_layers + (size_t)l * R.total_bwd,
                                      A.Rp, R, tape + T.hx + (size_t)l * num_atoms * (nf + H), num_atoms, nf, H,
                                      A.Lp, f32b);
    if (rc) return rc;
    if (hipEventRecord(ev(2 * l + 1), st2) != hipSuccess) return -2;
    if (serial && hipStreamWaitEvent(st, ev(2 * l + 1), 0) != hipSuccess) return -2;
  }
  if (n_layers > 0 && hipStreamWaitEvent(st, ev(1), 0) != hipSuccess) return -2;
  if (dequant_kind == ENFLOW_DEQUANT_ARGMAX && num_atoms > 0) {
    const int chunks = (num_atoms + 31) / 32;
    hipLaunchKernelGGL(chunk_ptr_kernel, dim3(chunks / BLOCK + 1), dim3(BLOCK), 0, st, num_atoms, chunks, chunk);
    const int rc = argmax_grads(st, Wl, ws + Wl.buf0, chunk, chunks, 32, H, nf, num_atoms, h_data, noise,
                                dequant_raw, adj_h, adj_ldj, grad_dequant);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(poison_on_err_kernel, dim3(64), dim3(256), 0, st, err_flag, grad_layers,
                     (long long)n_layers * R.total_bwd, dequant_kind == ENFLOW_DEQUANT_ARGMAX ? grad_dequant : nullptr,
                     (long long)(H * nf + H + 2 * nf * H + 2 * nf));
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int enflow_lf_backward_large_f32(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                                 const int32_t* mol_ptr, const float* r_cut, const float* box, const float* tape,
                                 const float* layers, const float* layers_bwd, const float* layers_raw, int n_layers,
                                 int dequant_kind, const float* dequant_raw, const float* h_data, const float* noise,
                                 float dt, float cw,
                                 float* adj_h, float* adj_g, float* adj_pos, float* adj_vel, const float* adj_ldj,
                                 float* grad_layers, float* grad_dequant,
                                 void* workspace, int64_t workspace_bytes, int64_t pair_row_bound,
                                 int32_t* err_flag, void* stream) {
  return lf_backward_large_impl(num_mols, num_atoms, max_mol_atoms, nf, H, mol_ptr, r_cut, box, tape, layers,
                                layers_bwd, layers_raw, n_layers, dequant_kind, dequant_raw, h_data, noise, dt, cw,
                                adj_h, adj_g, adj_pos, adj_vel, adj_ldj, grad_layers, grad_dequant, workspace,
                                workspace_bytes, pair_row_bound, err_flag, stream, nullptr, nullptr, nullptr);
}

// ---- standalone EGCL.forward backward ------------------------------------
// Workspace: the one-layer backward's, then scratch for the (unused) velocity /
// g adjoints and a zero log|detJ| adjoint.
static size_t egcl_bwd_extra(int num_atoms, int nf) {
  return al64((size_t)num_atoms * 3) + al64((size_t)num_atoms * nf) + 64;
}
int64_t enflow_egcl_backward_workspace_size(int num_mols, int num_atoms, int nf, int H, int64_t pair_row_bound) {
  if (num_mols < 0 || num_atoms < 0 || nf < 1 || nf > BWD_NFMAX || !hid_ok_b(H) || pair_row_bound < 0) return -1;
  return (int64_t)((bwd_ws(num_mols, num_atoms, nf, H, 1, pair_row_bound).total + egcl_bwd_extra(num_atoms, nf)) *
                   sizeof(float));
}

int enflow_egcl_backward_f32(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                             const int32_t* mol_ptr, const float* r_cut, const float* box,
                             const float* tape, const int32_t* pair_counts,
                             const float* layer, const float* layer_bwd, const float* layer_raw, int egcl_flags,
                             float cw, const float* adj_Q, const float* adj_F, const float* adj_G,
                             float* adj_h, float* adj_pos, float* grad_layer,
                             void* workspace, int64_t workspace_bytes, int64_t pair_row_bound,
                             int32_t* err_flag, void* stream) {
  if (num_mols < 0 || num_atoms < 0 || nf < 1 || nf > BWD_NFMAX || !hid_ok_b(H) || pair_row_bound < 0) return -1;
  if (!adj_Q || !adj_F || !adj_G || !workspace) return -1;
  const BwdWs Wl = bwd_ws(num_mols, num_atoms, nf, H, 1, pair_row_bound);
  if ((uint64_t)workspace_bytes < (Wl.total + egcl_bwd_extra(num_atoms, nf)) * sizeof(float)) return -6;
  float* extra = reinterpret_cast<float*>(workspace) + Wl.total;
  float* avel = extra;
  float* ag = avel + al64((size_t)num_atoms * 3);
  float* zero = ag + al64((size_t)num_atoms * nf);
  if (hipMemsetAsync(zero, 0, 64 * sizeof(float), SB(stream)) != hipSuccess) return -2;
  return lf_backward_impl(num_mols, num_atoms, max_mol_atoms, nf, H, mol_ptr, r_cut, box, tape, pair_counts, layer,
                          layer_bwd, layer_raw, 1, ENFLOW_DEQUANT_NONE | ((egcl_flags & 0xff) ? ENFLOW_EGCL_VARIANTS : 0) | (egcl_flags & ENFLOW_BWD_F32),
                          nullptr, nullptr, nullptr, 0.f, cw, adj_h, ag, adj_pos, avel, zero, grad_layer, nullptr,
                          workspace, workspace_bytes, pair_row_bound, err_flag, stream, adj_Q, adj_F, adj_G);
}

// molecules past 64 atoms: the large-system backward on a one-layer tape of
// enflow_lf_forward_large_f32 (dt 0, dequant NONE)
int64_t enflow_egcl_backward_large_workspace_size(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                                                  int64_t pair_row_bound) {
  const int64_t w = enflow_lf_backward_large_workspace_size(num_mols, num_atoms, max_mol_atoms, nf, H,
                                                            pair_row_bound);
  if (w < 0) return -1;
  return w + (int64_t)(egcl_bwd_extra(num_atoms, nf) * sizeof(float));
}

int enflow_egcl_backward_large_f32(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                                   const int32_t* mol_ptr, const float* r_cut, const float* box, const float* tape,
                                   const float* layer, const float* layer_bwd, const float* layer_raw,
                                   int egcl_flags, float cw, const float* adj_Q, const float* adj_F,
                                   const float* adj_G, float* adj_h, float* adj_pos, float* grad_layer,
                                   void* workspace, int64_t workspace_bytes, int64_t pair_row_bound,
                                   int32_t* err_flag, void* stream) {
  const int64_t w = enflow_lf_backward_large_workspace_size(num_mols, num_atoms, max_mol_atoms, nf, H,
                                                            pair_row_bound);
  if (w < 0 || !adj_Q || !adj_F || !adj_G || !workspace) return -1;
  if (workspace_bytes < w + (int64_t)(egcl_bwd_extra(num_atoms, nf) * sizeof(float))) return -6;
  float* extra = reinterpret_cast<float*>(static_cast<char*>(workspace) + w);
  float* avel = extra;
  float* ag = avel + al64((size_t)num_atoms * 3);
  float* zero = ag + al64((size_t)num_atoms * nf);
  if (hipMemsetAsync(zero, 0, 64 * sizeof(float), SB(stream)) != hipSuccess) return -2;
  return lf_backward_large_impl(num_mols, num_atoms, max_mol_atoms, nf, H, mol_ptr, r_cut, box, tape, layer,
                                layer_bwd, layer_raw, 1, ENFLOW_DEQUANT_NONE | ((egcl_flags & 0xff) ? ENFLOW_EGCL_VARIANTS : 0) | (egcl_flags & ENFLOW_BWD_F32),
                                nullptr, nullptr, nullptr, 0.f, cw, adj_h, ag, adj_pos, avel, zero, grad_layer,
                                nullptr, workspace, w, pair_row_bound, err_flag, stream, adj_Q, adj_F, adj_G);
}

// ---- standalone ArgMax.forward backward ------------------------------------
struct AmBwdWs { size_t apre, spre, anet, part, total; };
static AmBwdWs am_bwd_ws(int num_atoms, int nf, int H) {
  AmBwdWs W;
  size_t o = 0;
  const size_t A = (size_t)num_atoms;
  W.apre = o; o += al64(A * H);
  W.spre = o; o += al64(A * H);
  W.anet = o; o += al64(A * 2 * nf);
  const size_t cha = (size_t)cdiv(num_atoms, OA_CHUNK_ATOM);
  W.part = o; o += al64(cha * ((size_t)H * (nf + 1) + (size_t)2 * nf * (H + 1)));
  W.total = o;
  return W;
}
int64_t enflow_argmax_backward_workspace_size(int num_atoms, int nf, int H) {
  if (num_atoms < 0 || nf < 1 || nf > NFMAX || !hid_ok_b(H)) return -1;
  return (int64_t)(am_bwd_ws(num_atoms, nf, H).total * sizeof(float));
}

int enflow_argmax_backward_f32(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                               const int32_t* mol_ptr, const float* h, const float* dequant_raw, const float* noise,
                               const float* adj_z, const float* adj_log_q, float* grad_dequant,
                               void* workspace, int64_t workspace_bytes, void* stream) {
  if (num_mols < 0 || num_atoms < 0 || max_mol_atoms < 0 || max_mol_atoms > 64 || nf < 1 || nf > BWD_NFMAX ||
      !hid_ok_b(H))
    return -1;
  if (!mol_ptr || !h || !dequant_raw || !noise || !adj_z || !adj_log_q || !grad_dequant || !workspace) return -1;
  const AmBwdWs W = am_bwd_ws(num_atoms, nf, H);
  if ((uint64_t)workspace_bytes < W.total * sizeof(float)) return -6;
  if (num_mols == 0) return 0;
  hipStream_t st = SB(stream);
  float* ws = reinterpret_cast<float*>(workspace);
  float *apre = ws + W.apre, *spre = ws + W.spre, *anet = ws + W.anet;
#define CALL(HH, NN)                                                                                      \
  hipLaunchKernelGGL((argmax_bwd_kernel<HH, NN>), dim3(num_mols), dim3(BLOCK), 0, st, mol_ptr, nf, h,      \
                     noise, dequant_raw, adj_z, adj_log_q, apre, spre, anet)
  DISPATCH_HN_B(H, max_mol_atoms, CALL);
#undef CALL
  const int rW1 = 0, rb1 = H * nf, rW2 = rb1 + H, rb2 = rW2 + 2 * nf * H;
  OuterBatch ob;
  ob.nd = 0;
  int wg = 0;
  float* part = ws + W.part;
  add_desc(ob, wg, apre, H, H, h, nf, nf, nullptr, num_atoms, num_atoms, part, grad_dequant + rW1,
           grad_dequant + rb1);
  add_desc(ob, wg, anet, 2 * nf, 2 * nf, spre, H, H, nullptr, num_atoms, num_atoms, part, grad_dequant + rW2,
           grad_dequant + rb2);
  return run_outer(ob, wg, st);
}

}  // extern "C"
