// enflow_split.hip -- the feature-split latency instance of the fused flow
// (LFIntegrator.forward / reverse, enflow/flow/dynamics.py:10-37, driving
// EGCL.forward, enflow/nn/egcl.py:76-92) for batches that leave CUs idle: the
// stated 1024-molecule batch split over 8 GPUs is 128 molecules per GPU
// (enflow/main.py:141-143, DistributedSampler), a molecule per CU and half the
// CUs idle, so the step time is one molecule's serial chain of layers.
//
// What sets that chain in the whole-tile instances (phase stamps, profiles/r05):
// a wave owns a 32-pair edge tile and streams every H x H weight fragment of
// its three GEMMs from L2 (64 KB per GEMM per tile), one chain step ahead, so
// each F16X3 step waits on an L2 round trip; the tile loop is ~60 % of a layer.
//
// Here the eight waves of a workgroup share every tile and split its OUTPUT
// features over two pipeline stages: stage-A wave b (waves 0-3) owns features
// 32 b .. 32 b + 31 of edge_nn.0 and edge_nn.2, stage-B wave b (waves 4-7) the
// same features of coord_nn.0 and of the message sums (H = 128), so each wave's
// weight blocks (hi / lo fp16, 16-20 KB) are loaded into registers once per
// layer, during the pair build.  A GEMM's input (all 128 features of the 32
// pairs) is exchanged through LDS as the producers' own fp16 hi / lo split, in
// the MFMA B-operand lane layout (one ds_write_b128 / ds_read_b128 per lane and
// k-slice, conflict-free); two barriers per pipeline step (fs_edge_tiles).  Each
// stage-B wave segment-sums the messages of its own 32 features (selection-
// matrix MFMAs as in edge_tiles) and the four coord_nn.2 partial dots are added
// in block order (deterministic).  The node part is split the same way
// (fs_node_g, the vel_scaling_nn items in the tiles' first step).
//
// SPLIT = 2 (at most half as many molecules as CUs): two workgroups per
// molecule, on two CUs, each owning half of the molecule's rows.  Message and
// force sums are per row, so each workgroup's aggregates, node phase and
// leapfrog update of its own atoms are complete; the only exchange per layer is
// the updated positions and features of its atoms (what the partner's next
// neighbour list and edge_nn.0 inputs read: 3 + nf floats per atom), handed off
// as 8-byte {value, tag} granules written with `sc1` stores and polled with
// `sc1` loads (MI355X_MICROARCH.md: the data-tagged granule hand-off, ~1 us).
// The pair sits on one XCD (blocks b and b ^ 8); a bounded wait flags
// ENFLOW_ERR_HANDOFF and the host re-runs the launch on the whole-tile instance.
//
// Results are deterministic; they may differ from the whole-tile instances in
// the last bits (the coord_nn.2 dot is summed per 32-feature block first).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <mutex>
#include "enflow_hip.h"
#include "enflow_timing.h"
#include "enflow_split.h"

#define WAVES 8
// the message MFMAs read the group's operand image: no per-wave message image in Smem
#define ENFLOW_MSG_MFMA 0
namespace enflow_fs {
#include "flow_device.h"

constexpr int NMX = 32;                // molecule capacity (<= 32-atom molecules)
constexpr int HALF = NMX / 2;          // rows per workgroup of a SPLIT = 2 pair
constexpr int XG = NFMAX + 3;          // granules per atom in a hand-off: pos (3) + h (nf)
constexpr int XSLOT = HALF * XG;       // granules per (molecule, half, parity)

template <int H>
struct FsSmem {
  static constexpr int NT = H / 32, KS = 2 * NT;
  Smem<H, NMX, NMX> s;
  // GEMM operands, [k-slice][hi | lo][lane] x 16 B: edge_nn.2's (x0) and, per
  // tile parity, coord_nn.0's (e, also the messages)
  alignas(16) uint32_t xa[KS][2][64][4];
  alignas(16) uint32_t xe[2][KS][2][64][4];
  float phip[2][NT][32];               // coord_nn.2 partial dots [tile parity][block][pair]
  uint32_t tb[3][32];                  // per tile mod 3: selection words (f16 multiplicity << 16 | segment)
  int rt[3][96];                       // per tile mod 3: segment rows (slots 32.. absorb the non-start lanes)
  int nseg[3];
  int dat[2][32];                      // per tile parity: pair's row atom | column atom << 8
  float rad[2][32];                    // per tile parity: pair's radial
  alignas(16) float fx[3][32][4];      // per tile mod 3: pair's coord_diff (x, y, z), multiplicity
  int frow[3][32];                     // per tile mod 3: pair's row, -1 - lane past the pairs
  alignas(16) float dummy[NT][32];     // message row of lanes without a segment (per stage-B wave)
  // node biases per layer parity, the packed layer's contiguous run from bn1:
  // node_nn.0 bias, vel_scaling_nn.0 bias, vel_scaling_nn.2 weight (H each),
  // node_nn.2 bias (NFMAX), vel_scaling_nn.2 bias
  static constexpr int NB = 3 * H + NFMAX + 1;
  alignas(16) float nb[2][(NB + 3) & ~3];
  int timeout;
};

struct FsArgs {
  uint64_t* xch;       // [mols][2 halves][2 parities][XSLOT] hand-off granules (SPLIT = 2)
  uint32_t* ctl;       // [0] ticket, [1] epoch (+1 per launch, by the last workgroup)
  float* part;         // [blocks] log|detJ| partial per workgroup
  int split;           // 1 or 2
  int blocks;
  int spin_limit;      // polls per hand-off wait before ENFLOW_ERR_HANDOFF (enflow_set_handoff_spin_limit)
};

// one hand-off wait (SPLIT = 2): poll the partner's granule until it carries
// `tag`, at most `limit` polls; a wait that gives up sets F.timeout, and once
// set every later wait of the workgroup gives up after its first poll, so a
// lost partner costs one bounded wait per workgroup, not one per granule and
// layer.  limit 0 gives up without polling (the forced ENFLOW_ERR_HANDOFF path).
template <class FS>
__device__ __forceinline__ uint64_t fs_poll(FS& F, const uint64_t* slot, uint32_t tag, int limit) {
  uint64_t g = 0;
  for (int spins = 0;; ++spins) {
    if (spins >= limit) {
      F.timeout = 1;
      break;
    }
    g = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(g >> 32) == tag) break;
    if (*reinterpret_cast<volatile int*>(&F.timeout)) break;
    __builtin_amdgcn_s_sleep(1);
  }
  return g;
}

// the wave's weight blocks (F16X3 fragments, registers): stage A (waves
// 0 .. NT - 1) block b of edge_nn.0 and edge_nn.2, stage B block b of coord_nn.0
template <int H>
struct FsW {
  static constexpr int NT = H / 32, KS = 2 * NT;
  f32x4 g0h[KS0MAX], g0l[KS0MAX], wh[KS], wl[KS];
  f32x4 qh, ql;   // stage B: vel_scaling_nn.0 block b (its item runs in the tiles' first step)
  // in three parts (part 0: edge_nn.0 and k-slices 0 .. 2, part 1: 3 .. 5, part
  // 2: the rest), requested between the steps of the pair build: the CU's load
  // path (~144 KB per layer) drains beside the build's LDS work instead of
  // stalling the issuing waves at one point
  __device__ __forceinline__ void load(rsrc_t W, const EgclLayout& L, int lane, int w, int ks0, int part) {
    const int vo = lane * 32, b = w % NT;
    const bool A = w < NT;
    const int t0 = part == 0 ? 0 : (part == 1 ? 3 : 6), t1 = part == 0 ? 3 : (part == 1 ? 6 : KS);
    if (!A && part == 0) {
      qh = bload4(W, vo, (L.wv1x + b * 512) * 4);
      ql = bload4(W, vo + 16, (L.wv1x + b * 512) * 4);
    }
    if (A && part == 0) {
#pragma unroll
      for (int ks = 0; ks < KS0MAX; ++ks) {
        if (ks < ks0) {
          g0h[ks] = bload4(W, vo, (L.we1x + (b * KS0MAX + ks) * 512) * 4);
          g0l[ks] = bload4(W, vo + 16, (L.we1x + (b * KS0MAX + ks) * 512) * 4);
        }
      }
    }
    const int off = A ? L.we2x : L.wc1x;
#pragma unroll
    for (int ts = 0; ts < KS; ++ts) {
      if (ts >= t0 && ts < t1) {
        wh[ts] = bload4(W, vo, (off + (b * KS + ts) * 512) * 4);
        wl[ts] = bload4(W, vo + 16, (off + (b * KS + ts) * 512) * 4);
      }
    }
  }
};

// accumulator of output block w from the LDS bias image (feature 32 w + 8 g4 + 4 hh + u)
__device__ __forceinline__ f32x16 bias_block(const float* __restrict__ b, int w, int hh) {
  f32x16 a;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const f32x4 v = ld4(b + 32 * w + 8 * g4 + 4 * hh);
#pragma unroll
    for (int u = 0; u < 4; ++u) a[4 * g4 + u] = v[u];
  }
  return a;
}
__device__ __forceinline__ void silu_block(f32x16& X, float c, float K) {
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const f32x4 y = silu4s((f32x4){X[4 * g4], X[4 * g4 + 1], X[4 * g4 + 2], X[4 * g4 + 3]}, c, K);
#pragma unroll
    for (int u = 0; u < 4; ++u) X[4 * g4 + u] = y[u];
  }
}
__device__ __forceinline__ void st_u4(uint32_t* p, const f16x8& v) {
  *reinterpret_cast<u32x4v*>(p) = __builtin_bit_cast(u32x4v, v);
}
__device__ __forceinline__ f16x8 ld_u4(const uint32_t* p) {
  return __builtin_bit_cast(f16x8, *reinterpret_cast<const u32x4v*>(p));
}

// A layer's bias images, one element of each per thread (BLOCK = 4 H): the
// tile biases in edge_tiles' order and scale (be1 K0, be2 K1, bc1 K2, wc2) and
// the node biases (FsSmem::nb).  Requested in registers during the previous
// layer's node items, stored to LDS after them: no L2 round trip on a phase.
struct FsBias {
  float t, n;
};
// (Both images are contiguous runs of the packed layer, egcl_layout: be1 be2 bc1
// wc2, and bn1 bv1 wv2 bn2 bv2 -- no per-thread choice between layout fields,
// which the compiler would turn into a dynamically indexed copy of the layout
// in scratch.)
template <int H>
__device__ __forceinline__ FsBias fs_bias_load(const float* __restrict__ Lp, const EgclLayout& L, int tid) {
  static_assert(BLOCK == 4 * H, "one tile-bias element per thread");
  FsBias r;
  r.t = Lp[L.be1 + tid];
  r.n = tid < FsSmem<H>::NB ? Lp[L.bn1 + tid] : 0.f;
  return r;
}
template <int H>
__device__ __forceinline__ void fs_bias_store(FsSmem<H>& F, const float* __restrict__ Lp, const EgclLayout& L, int tid,
                                              const FsBias& r, int par) {
  const int g = tid / H;
  const float K = g == 0 ? Lp[L.scl + 4] : (g == 1 ? Lp[L.scl + 0] : (g == 2 ? Lp[L.scl + 2] : 1.f));
  F.s.bias[tid] = r.t * K;
  if (tid < FsSmem<H>::NB) F.nb[par][tid] = r.n;
}

// node_nn (egcl.py:51-54, 65-67) on the workgroup's rows with node_phase_x3_f's
// arithmetic: wave tp < NT the item of features 32 tp .. (G partials:
// node_nn.0 over [h, agg], act, node_nn.2).  (The vel_scaling_nn items run in
// the edge tiles' first step, fs_edge_tiles.)  nb: the layer's node biases
// (FsSmem::nb).
template <int H>
__device__ __forceinline__ void fs_node_g(FsSmem<H>& F, const float* __restrict__ Lp, const EgclLayout& L,
                                              int tid, int r0, int rb, int nf, const float* __restrict__ nb
                                              STAMP_ARGS) {
  constexpr int NT = H / 32, KS = H / 16;
  constexpr int AST = Smem<H, NMX, NMX>::AST;
  auto& sm = F.s;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hh = lane >> 5, tp = w % NT, vo = lane * 32;
  const rsrc_t W = weights_rsrc(Lp, L.total);
  const int a = j;                        // row within the workgroup's block
  const bool va = a < rb;
  const int ag = r0 + (va ? a : 0);
  const uint32_t vm = va ? ENFLOW_BIG_BITS : 0u;
  uint32_t bigw = 0u;
  {   // ---- node_nn item tp
    const f32x4 nh = bload4(W, vo, (L.wn1hx + tp * 512) * 4), nl = bload4(W, vo + 16, (L.wn1hx + tp * 512) * 4);
    f32x4 gfh[2], gfl[2], ah[KS], al[KS];
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
    const float inv_n1 = Lp[L.scl + 9], inv_n2 = Lp[L.scl + 11];
    f32x16 hin;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) hin[jj] = (va && 8 * hh + jj < nf) ? sm.h[ag * NFP + 8 * hh + jj] : 0.f;
    f16x8 hh16, hl16;
    split_f16(hin, 0, hh16, hl16);
    uint32_t oa = or_hi(0u, hh16), on = 0u;
    STAMP(16);
    f32x16 acc = (f32x16)0.f;
    acc = mfma_f16(nh, hh16, acc);
    acc = mfma_f16(nh, hl16, acc);
    acc = mfma_f16(nl, hh16, acc);
    const float* arow = &sm.agg[(va ? a : 0) * AST];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      f32x16 av;
      const f32x4 a0 = ld4(arow + 16 * ks + 8 * hh), a1 = ld4(arow + 16 * ks + 8 * hh + 4);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        av[jj] = va ? a0[jj] : 0.f;
        av[4 + jj] = va ? a1[jj] : 0.f;
      }
      f16x8 bh, bl;
      split_f16(av, 0, bh, bl);
      oa = or_hi(oa, bh);
      acc = mfma_f16(ah[ks], bh, acc);
      acc = mfma_f16(ah[ks], bl, acc);
      acc = mfma_f16(al[ks], bh, acc);
    }
    STAMP(17);
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 b1 = ld4(nb + 32 * tp + 8 * g4 + 4 * hh);   // node_nn.0 bias
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[4 * g4 + u] = silu_f(fmaf(acc[4 * g4 + u], inv_n1, b1[u]));
    }
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
    bigw = (__ballot((oa & vm) != 0u) ? (uint32_t)BIGK_HA : 0u) | (__ballot((on & vm) != 0u) ? (uint32_t)BIGK_NH : 0u);
    if (va) {
#pragma unroll
      for (int r = 0; r < NFMAX / 2; ++r) {
        const int q = rho(r, hh);
        if (q < nf) sm.u.nd.gp[tp][q][a] = gacc[r] * inv_n2;
      }
    }
    STAMP(18);
  }
  if (lane == 0) atomicOr(&sm.big, bigw | (uint32_t)BIGK_NODE);
}

// forces of one tile (egcl.py:68-74: trans = clamp(coord_diff * phi), segment
// sums for the mean), phi = the four partial dots in block order, the pair's
// coord_diff / multiplicity / row from its decode (FsSmem::fx, frow); run by one
// stage-B wave, tiles in order (rows continuing into the next tile accumulate)
template <int H>
__device__ __forceinline__ void tile_forces(FsSmem<H>& F, int P, int tile, int lane, bool& range_bad) {
  constexpr int NT = H / 32;
  constexpr int AST = Smem<H, NMX, NMX>::AST;
  auto& sm = F.s;
  const int j = lane & 31, hh = lane >> 5, t3 = tile % 3;
  const bool valid = tile * 32 + j < P;
  const f32x4 d = ld4(&F.fx[t3][j][0]);
  const int row = F.frow[t3][j];
  float phi = 0.f;
#pragma unroll
  for (int b = 0; b < NT; ++b) phi += F.phip[tile & 1][b][j];
  range_bad |= valid && !__builtin_isfinite(phi);
  const SegExec SE = seg_exec(row);
  const int row_next = __shfl_down(row, 1, 32);
  const bool seg_end = valid && (j == 31 || row_next != row);
  f32x4* const fslot = reinterpret_cast<f32x4*>(&sm.agg[(valid ? row : 0) * AST + H]);   // H + 3: padding
  const f32x4 fold = *fslot;
  float tx = d[3] * clamp100(d[0] * phi);
  float ty = d[3] * clamp100(d[1] * phi);
  float tz = d[3] * clamp100(d[2] * phi);
  float tw = 0.f;
  seg_scan4x(tx, ty, tz, tw, SE);
  if (seg_end && hh == 0) *fslot = fold + (f32x4){tx, ty, tz, tw};
}

// EGCL edge part of the workgroup's rows (edge_tiles' contract: agg[row][0..H)
// message sums, agg[row][H..H+2] force sums, multiplicity-weighted) as a
// two-stage pipeline over the tiles.  Waves 0..3 (stage A) own output block b
// of edge_nn.0 and edge_nn.2, waves 4..7 (stage B) block b of coord_nn.0 and
// of the message sums: each keeps one weight block in registers, and the two
// waves on a SIMD (one per stage) run different phases side by side.  Step s:
//   A: GEMM0, act, operand split of tile s   | B: GEMM2, act, coord_nn.2 partial
//                                            |    dot of tile s - 1
//   -- barrier --
//   A: GEMM1, act, operand split of tile s   | B: message MFMAs of tile s - 1; forces
//      (-> e image, double-buffered)         |    of tile s - 1 (one wave); pair decode
//                                            |    + segment tables of tile s + 1 (another)
//   -- barrier --
// Each wave handles every tile in order, so message and force rows that
// continue into the next tile accumulate in order: deterministic.
// KS0: edge_nn.0 k-slices compiled (gemm0_ksteps(nf) <= KS0; slices past it
// multiply zero fragments by zero inputs: exact).
template <int H, int KS0>
__device__ __forceinline__ void fs_edge_tiles(FsSmem<H>& F, const float* __restrict__ Lp, const EgclLayout& L,
                                              const MolRef& M, int nf, int tid, int r0, int rb, const FsW<H>& Wt,
                                              const float* __restrict__ nb STAMP_ARGS) {
  constexpr int NT = H / 32, KS = 2 * NT;
  constexpr int AST = Smem<H, NMX, NMX>::AST;
  auto& sm = F.s;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool stA = w < NT;                   // stage
  const int b = w % NT;                      // output block
  const int j = lane & 31, hh = lane >> 5;
  const int P = sm.npairs;
  const int T = (P + 31) >> 5;
  // (the caller zeroed agg and staged the layer's bias image before the pair build)
  const float K0 = Lp[L.scl + 4], K1 = Lp[L.scl + 0], K2 = Lp[L.scl + 2];
  constexpr float NLOG2E = -1.4426950408889634f;
  const float c0 = NLOG2E * Lp[L.scl + 5], c1 = NLOG2E * Lp[L.scl + 1], c2 = NLOG2E * Lp[L.scl + 3];
  const int nch = gemm0_nch(nf);
  const bool rad7 = gemm0_radial_slot7(nf);
  // the transposed (pairs x features) reads of block b's message operand from
  // the e image (ds_read_b64_tr_b16: lane 4q + p of each 16-lane group
  // addresses pair q, features 4p .. 4p + 3 of its 16-feature half)
  const int tr_off = (8 * hh + ((lane >> 2) & 3) + 32 * (lane & 1)) * 4 + 2 * ((lane >> 1) & 1);
  bool range_bad = false;
  uint32_t bigw = 0u;
  // stage B: a tile's pair decode (atoms, radial) and segment tables -> LDS
  auto decode = [&](int tile) {
    const int p = tile * 32 + j;
    const bool valid = p < P;
    uint32_t pr = sm.pairs[valid ? p : 0];
    pr = valid ? pr : 0u;
    const int il = (int)(pr & 0xffu), jl = (int)((pr >> 8) & 0xffu), i = r0 + il;
    const float c = (float)(pr >> 16);
    const int row = valid ? il : -1 - j;
    const float dx = pbc1(sm.pos[i * 3 + 0] - sm.pos[jl * 3 + 0], M.bx * 0.5f);
    const float dy = pbc1(sm.pos[i * 3 + 1] - sm.pos[jl * 3 + 1], M.by * 0.5f);
    const float dz = pbc1(sm.pos[i * 3 + 2] - sm.pos[jl * 3 + 2], M.bz * 0.5f);
    const int par = tile & 1, tpar = tile % 3;
    const int row_prev = __shfl_up(row, 1, 32);
    const bool start = j == 0 || row_prev != row;
    const uint32_t Sb = (uint32_t)__ballot(start);
    const int seg = __builtin_popcount(Sb & (uint32_t)((2ull << j) - 1ull)) - 1;
    F.tb[tpar][j] = ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)c) << 16) | (uint32_t)seg;
    F.rt[tpar][(start && hh == 0) ? seg : 32 + lane] = valid ? il : -1;
    F.nseg[tpar] = __builtin_popcount(Sb);
    F.dat[par][j] = i | (jl << 8);
    F.rad[par][j] = dx * dx + dy * dy + dz * dz;   // egcl.py:79
    const int t3 = tile % 3;
    st4(&F.fx[t3][j][0], (f32x4){dx, dy, dz, c});
    F.frow[t3][j] = row;
  };
  if (!stA && b == 0 && T > 0) decode(0);
  __syncthreads();
  STAMP(9);
  for (int s = 0; s <= T; ++s) {
    if (stA) {
      if (s < T) {   // ---- GEMM0 (egcl.py:57-58) of tile s, block b; act, operand split
        const int par = s & 1;
        const bool valid = s * 32 + j < P;
        const int at = F.dat[par][j];
        const int i = at & 0xff, jl = at >> 8;
        const float radial = F.rad[par][j];
        const uint32_t vmask = valid ? ENFLOW_BIG_BITS : 0u;
        f32x16 x0 = bias_block(sm.bias, b, hh);
        uint32_t o0 = 0u;
#pragma unroll
        for (int ks = 0; ks < KS0; ++ks) {
          f32x16 in;
          const float* hrow = &sm.h[(hh ? jl : i) * NFP + 8 * (ks < nch ? ks : 0)];   // rows zero-padded past nf
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) in[jj] = ks < nch ? hrow[jj] : 0.f;
          in[7] = (hh && ks == nch - 1 && rad7) ? radial : in[7];
          in[0] = (hh == 0 && ks == nch && !rad7) ? radial : in[0];
          f16x8 bh, bl;
          split_f16(in, 0, bh, bl);
          o0 = or_hi(o0, bh);
          x0 = mfma_f16(Wt.g0h[ks], bh, x0);
          x0 = mfma_f16(Wt.g0h[ks], bl, x0);
          x0 = mfma_f16(Wt.g0l[ks], bh, x0);
        }
        bigw |= __ballot((o0 & vmask) != 0u) ? (uint32_t)BIGK_X0 : 0u;
        silu_block(x0, c0, K0);
        uint32_t o1 = 0u;
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          f16x8 bh, bl;
          split_f16(x0, sl, bh, bl);
          o1 = or_hi(o1, bh);
          st_u4(&F.xa[2 * b + sl][0][lane][0], bh);
          st_u4(&F.xa[2 * b + sl][1][lane][0], bl);
        }
        bigw |= __ballot((o1 & vmask) != 0u) ? (uint32_t)BIGK_Y0 : 0u;
      }
    } else if (s > 0) {   // ---- GEMM2 (egcl.py:35-42) of tile s - 1, block b; coord_nn.2 partial dot
      const int par = (s - 1) & 1;
      const auto& xe = F.xe[par];
      f32x16 hc = bias_block(sm.bias + 2 * H, b, hh);
#pragma unroll
      for (int ts = 0; ts < KS; ++ts) {
        const f16x8 bh = ld_u4(&xe[ts][0][lane][0]), bl = ld_u4(&xe[ts][1][lane][0]);
        hc = mfma_f16(Wt.wh[ts], bh, hc);
        hc = mfma_f16(Wt.wh[ts], bl, hc);
        hc = mfma_f16(Wt.wl[ts], bh, hc);
      }
      float part = 0.f;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 w2 = ld4(sm.bias + 3 * H + 32 * b + 8 * g4 + 4 * hh);
        const f32x4 y = silu4s((f32x4){hc[4 * g4], hc[4 * g4 + 1], hc[4 * g4 + 2], hc[4 * g4 + 3]}, c2, K2);
#pragma unroll
        for (int u = 0; u < 4; ++u) part += w2[u] * y[u];
      }
      part += __shfl_xor(part, 32, 64);
      F.phip[par][b][j] = part;   // both lane halves: the same value to the same word
    } else {   // ---- step 0: vel_scaling_nn item b (egcl.py:26-30, 62-64; depends on h only)
      // node_phase_x3_f's arithmetic: Q partial over features 32 b .. of the rows
      // (lane j = row j), summed with the other items in the tail
      const bool va = j < rb;
      const int ag = r0 + (va ? j : 0);
      f32x16 hin;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) hin[jj] = (va && 8 * hh + jj < nf) ? sm.h[ag * NFP + 8 * hh + jj] : 0.f;
      f16x8 hh16, hl16;
      split_f16(hin, 0, hh16, hl16);
      const uint32_t oh = or_hi(0u, hh16);
      f32x16 acc = (f32x16)0.f;
      acc = mfma_f16(Wt.qh, hh16, acc);
      acc = mfma_f16(Wt.qh, hl16, acc);
      acc = mfma_f16(Wt.ql, hh16, acc);
      const float inv_v1 = Lp[L.scl + 7];
      float part = 0.f;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int f0 = 32 * b + 8 * g4 + 4 * hh;
        const f32x4 b1 = ld4(nb + H + f0), w2 = ld4(nb + 2 * H + f0);   // vel_scaling_nn.0 bias, .2 weight
#pragma unroll
        for (int u = 0; u < 4; ++u) part += w2[u] * silu_f(fmaf(acc[4 * g4 + u], inv_v1, b1[u]));
      }
      part += __shfl_xor(part, 32, 64);
      if (hh == 0 && va) sm.u.nd.qp[b][j] = part;
      const uint32_t vm = va ? ENFLOW_BIG_BITS : 0u;
      const uint32_t qb = __ballot((oh & vm) != 0u) ? (uint32_t)BIGK_HV : 0u;
      if (lane == 0) atomicOr(&sm.big, qb | (uint32_t)BIGK_NODE);
    }
    STAMP(10);
    __syncthreads();   // x0 of tile s, phi partials of tile s - 1 complete
    STAMP(11);
    if (stA) {
      if (s < T) {   // ---- GEMM1: edge_nn.2 (egcl.py:20-24) of tile s, block b; act, split -> e image
        const int par = s & 1;
        f32x16 e = bias_block(sm.bias + H, b, hh);
#pragma unroll
        for (int ts = 0; ts < KS; ++ts) {
          const f16x8 bh = ld_u4(&F.xa[ts][0][lane][0]), bl = ld_u4(&F.xa[ts][1][lane][0]);
          e = mfma_f16(Wt.wh[ts], bh, e);
          e = mfma_f16(Wt.wh[ts], bl, e);
          e = mfma_f16(Wt.wl[ts], bh, e);
        }
        STAMP(12);
        silu_block(e, c1, K1);
        uint32_t o2 = 0u;
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          f16x8 bh, bl;
          split_f16(e, sl, bh, bl);
          o2 = or_hi(o2, bh);
          st_u4(&F.xe[par][2 * b + sl][0][lane][0], bh);
          st_u4(&F.xe[par][2 * b + sl][1][lane][0], bl);
        }
        const uint32_t vmask = s * 32 + j < P ? ENFLOW_BIG_BITS : 0u;
        bigw |= __ballot((o2 & vmask) != 0u) ? (uint32_t)BIGK_M : 0u;
      }
    } else {
      if (s > 0) {   // message MFMAs of tile s - 1, block b
        const int par = (s - 1) & 1, tpar = (s - 1) % 3;
        const auto& xe = F.xe[par];
        // message segment sums of block b on the matrix cores (edge_tiles' MMA path):
        // agg[row(n)][32 b + f] += sum_p E[p][f] S[p][n], S[p][n] = multiplicity of p in segment n
        u32x4v tq[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          tq[qq] = *reinterpret_cast<const u32x4v*>(&F.tb[tpar][16 * (qq >> 1) + 8 * hh + 4 * (qq & 1)]);
        const int rn = F.rt[tpar][j];
        const int nseg = F.nseg[tpar];
        f16x8 sel[2];
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
        const bool vn = j < nseg && rn >= 0;
        float* const dstn = vn ? &sm.agg[rn * AST + 32 * b] : &F.dummy[b][0];
        s16x4 ar[4][2];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int rd = 0; rd < 2; ++rd)
            ar[k][rd] = lds_tr16(&xe[2 * b + ((lane >> 4) & 1)][k & 1][0][0] + tr_off + (16 * (k >> 1) + 4 * rd) * 4);
        f32x16 Y;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 v = ld4(dstn + 8 * g4 + 4 * hh);
#pragma unroll
          for (int u = 0; u < 4; ++u) Y[4 * g4 + u] = v[u];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(cat_f16x8(ar[k][0], ar[k][1]), sel[k >> 1], Y, 0, 0, 0);
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          st4(dstn + 8 * g4 + 4 * hh, (f32x4){Y[4 * g4], Y[4 * g4 + 1], Y[4 * g4 + 2], Y[4 * g4 + 3]});
      }
      if (s > 0 && b == (s - 1) % NT) tile_forces(F, P, s - 1, lane, range_bad);
      if (s + 1 < T && b == s % NT) decode(s + 1);
    }
    STAMP(13);
    __syncthreads();   // e of tile s, forces of tile s - 1, decode of tile s + 1 complete
    STAMP(14);
  }
  if (__ballot(range_bad))
    if (lane == 0) atomicOr(&sm.err, ENFLOW_ERR_RANGE);
  if (lane == 0 && T > 0) atomicOr(&sm.big, bigw | (uint32_t)BIGK_EDGE);
  __syncthreads();
  STAMP(15);
}

// ArgMax.forward (argmax.py:13-25) on the molecule: argmax_dequant's
// arithmetic, every atom (both workgroups of a pair draw the same noise
// elements, so their h agree bitwise); returns log_q of this thread's atoms.
// (argmax_dequant itself is reused as is.)

// the hand-off (SPLIT = 2): tag of (launch epoch, layer); never 0 (a zeroed slot never matches)
__device__ __forceinline__ uint32_t xtag(uint32_t epoch, int l) {
  return ((epoch & 0xffffffu) << 8) | 0x80u | (uint32_t)(l & 0x7f);
}
// publish the workgroup's atoms [r0, r0 + rb): pos (3) and h (nf), sc1 stores
template <int H>
__device__ __forceinline__ void fs_publish(FsSmem<H>& F, uint64_t* slot, int r0, int rb, int nf, uint32_t tag) {
  auto& sm = F.s;
  const int per = 3 + nf;
  for (int e = threadIdx.x; e < rb * per; e += BLOCK) {
    const int a = e / per, k = e - a * per;
    const float v = k < 3 ? sm.pos[(r0 + a) * 3 + k] : sm.h[(r0 + a) * NFP + (k - 3)];
    const uint64_t g = ((uint64_t)tag << 32) | (uint64_t)__float_as_uint(v);
    __hip_atomic_store(slot + a * XG + k, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// wait for the partner's atoms [r0, r0 + rb) of this tag (bounded: fs_poll, then ENFLOW_ERR_HANDOFF)
template <int H>
__device__ __forceinline__ void fs_consume(FsSmem<H>& F, const uint64_t* slot, int r0, int rb, int nf, uint32_t tag,
                                           int limit) {
  auto& sm = F.s;
  const int per = 3 + nf;
  for (int e = threadIdx.x; e < rb * per; e += BLOCK) {
    const int a = e / per, k = e - a * per;
    const uint64_t g = fs_poll(F, slot + a * XG + k, tag, limit);
    const float v = __uint_as_float((uint32_t)g);
    if (k < 3) sm.pos[(r0 + a) * 3 + k] = v;
    else sm.h[(r0 + a) * NFP + (k - 3)] = v;
  }
  __syncthreads();
}

template <int H, bool REV, int SPLIT, int KS0>
__global__ void __launch_bounds__(BLOCK, 1) lf_fs_kernel(FlowArgs A, FsArgs X) {
  __shared__ FsSmem<H> F;
  auto& sm = F.s;
  const int tid = threadIdx.x;
  STAMP_DECL
  const int b = blockIdx.x;
  // SPLIT = 2: blocks b and b ^ 8 (one XCD under round-robin placement) are the
  // two halves of molecule (b >> 4) * 8 + (b & 7)
  const int m = SPLIT == 2 ? (b >> 4) * 8 + (b & 7) : b;
  const int half = SPLIT == 2 ? (b >> 3) & 1 : 0;
  float ldj = 0.f;
  bool active = m < A.num_mols;
  MolRef M{0, 0, 0.f, 0.f, 0.f, 0.f};
  if (active) {
    M.a0 = A.mol_ptr[m];
    M.n = A.mol_ptr[m + 1] - M.a0;
    if (M.n > NMX || A.nf > NFMAX) {
      if (tid == 0) {
        const int e = M.n > NMX ? ENFLOW_ERR_TOO_MANY_ATOMS : ENFLOW_ERR_TOO_MANY_FEATURES;
        atomicOr(A.err, e);
        if (A.mol_err && half == 0) atomicOr(&A.mol_err[m], e);
      }
      active = false;
    }
  }
  if (active) {
    const int n = M.n, nf = A.nf;
    M.rc = A.r_cut[m];
    for (int e = tid; e < n * 3; e += BLOCK) {
      sm.pos[e] = (A.pos_in ? A.pos_in : A.pos)[(size_t)M.a0 * 3 + e];
      sm.vel[e] = (A.vel_in ? A.vel_in : A.vel)[(size_t)M.a0 * 3 + e];
      sm.boxa[e] = A.box[(size_t)M.a0 * 3 + e];
    }
    const float* const hin = A.h_in ? A.h_in : A.h;
    const float* const gin = A.g_in ? A.g_in : A.g;
    for (int e = tid; e < n * NFP; e += BLOCK) {   // rows zero-padded past nf
      const int a = e / NFP, q = e - a * NFP;
      const size_t src = (size_t)(M.a0 + a) * nf + q;
      sm.h[e] = q < nf ? hin[src] : 0.f;
      sm.g[e] = q < nf ? gin[src] : 0.f;
    }
    if (tid == 0) {
      sm.err = 0;
      sm.big = 0u;
      F.timeout = 0;
    }
    __syncthreads();
    if (n > 0) {
      M.bx = sm.boxa[0];
      M.by = sm.boxa[1];
      M.bz = sm.boxa[2];
    }
    // the workgroup's rows
    const int n0 = SPLIT == 2 ? (n + 1) >> 1 : n;
    const int r0 = half ? n0 : 0, rb = half ? n - n0 : n0;
    const int pr0 = half ? 0 : n0, prb = half ? n0 : n - n0;   // the partner's rows
    const uint32_t epoch = SPLIT == 2 ? __hip_atomic_load(&X.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    uint64_t* const xmine = SPLIT == 2 ? X.xch + ((size_t)(m * 2 + half) * 2) * XSLOT : nullptr;
    const uint64_t* const xpart = SPLIT == 2 ? X.xch + ((size_t)(m * 2 + (half ^ 1)) * 2) * XSLOT : nullptr;
    auto pbox = [&](int a, int d) { return sm.boxa[a * 3 + d]; };

    STAMP(0);
    if (!REV) {
      if (A.lq_mol != nullptr && half == 0 && tid == 0) ldj += A.lq_mol[m];   // dequantised ahead (dequant_kernel)
      if (A.dequant_kind == ENFLOW_DEQUANT_ARGMAX) {
        // every atom in both halves (the same draws); half 0 counts log_q
        const float lq = argmax_dequant<H, NMX, NMX, false, true>(sm, A.dequant, A.noise_src(), M.a0, n, nf);
        if (half == 0) ldj += lq;
      } else if (A.dequant_kind == ENFLOW_DEQUANT_FLOOR) {
        for (int e = tid; e < n * nf; e += BLOCK) {
          const int a = e / nf, q = e - a * nf;
          sm.h[a * NFP + q] += A.dequant_scale * A.noise_src().uniform((size_t)M.a0 * nf + e);
        }
        __syncthreads();
      }
    }

    STAMP(1);
    // Layer l: pair build (the layer's weight blocks requested beside it), edge
    // tiles (vel_scaling_nn in their first step), then the tail: T1 the node_nn
    // items beside the position update, the positions published as they are
    // updated and the partner's read, the next layer's bias images requested;
    // T2 the features' update, published.  The partner's
    // features are read just before the next layer's tiles, a pair build after
    // they were published: the hand-off latencies sit behind the node items and
    // the pair build (SPLIT = 2).  Reverse folds the next layer's half-step
    // (dynamics.py:28-30) into the tail.  Layer 0's biases and reverse half-step
    // are set up here.
    {
      const EgclLayout L0 = egcl_layout(H, nf);
      const float* Lp0 = A.layers + (size_t)(REV ? A.n_layers - 1 : 0) * L0.total;
      fs_bias_store(F, Lp0, L0, tid, fs_bias_load<H>(Lp0, L0, tid), 0);
      if (REV) {   // dynamics.py:28-30 on the workgroup's atoms, first layer
        for (int a = r0 + tid; a < r0 + rb; a += BLOCK) {
          for (int q = 0; q < nf; ++q) sm.h[a * NFP + q] -= sm.g[a * NFP + q] * A.dt;
          for (int d = 0; d < 3; ++d)
            sm.pos[a * 3 + d] = pbc1(sm.pos[a * 3 + d] - sm.vel[a * 3 + d] * A.dt, pbox(a, d));
        }
        __syncthreads();
        if constexpr (SPLIT == 2) {
          const uint32_t tag = xtag(epoch, 0x7f);
          fs_publish(F, xmine + XSLOT, r0, rb, nf, tag);
          fs_consume(F, xpart + XSLOT, pr0, prb, nf, tag, X.spin_limit);
        }
      }
    }
    constexpr int AST = Smem<H, NMX, NMX>::AST;
    for (int it = 0; it < A.n_layers; ++it) {
      int nfl = __builtin_amdgcn_readfirstlane(A.nf), nl = __builtin_amdgcn_readfirstlane(M.n), tid_l = tid;
      asm volatile("" : "+s"(nfl), "+s"(nl), "+v"(tid_l));
      MolRef Ml = M;
      Ml.n = nl;
      const EgclLayout L = egcl_layout(H, nfl);
      const int l = REV ? A.n_layers - 1 - it : it;
      const bool more = it + 1 < A.n_layers;
      const float* Lp = A.layers + (size_t)l * L.total;
      const float* Lpn = A.layers + (size_t)(REV ? l - 1 : l + 1) * L.total;   // next layer (valid when more)
      const int lane = tid_l & 63, w = __builtin_amdgcn_readfirstlane(tid_l >> 6);
      for (int e = tid_l; e < rb * AST; e += BLOCK) sm.agg[e] = 0.f;
      // the partner's features from the previous layer's tail: granule loads issued
      // here, their tags checked before the tiles (the load latency behind the pair
      // build; a granule not yet published is polled then)
      uint64_t hg = 0;
      const int he = tid_l;                 // one granule per thread: prb * nf <= 16 * NFMAX <= BLOCK
      const bool hget = SPLIT == 2 && it > 0 && he < prb * nfl;
      if (hget) {
        const int a = he / nfl, q = he - a * nfl;
        hg = __hip_atomic_load(xpart + ((it - 1) & 1) * XSLOT + a * XG + 3 + q, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      }
      STAMP(2);
      // this wave's weight blocks of the layer, requested in parts during the pair build
      FsW<H> Wt;
      const rsrc_t Wr = weights_rsrc(Lp, L.total);
      Wt.load(Wr, L, lane, w, KS0, 0);
      build_images(sm, Ml, tid_l);
      STAMP(3);
      Wt.load(Wr, L, lane, w, KS0, 1);
      block_counts(sm, Ml, tid_l, r0, rb, true);   // build_images zeroed the whole count matrix
      Wt.load(Wr, L, lane, w, KS0, 2);
      block_compact(sm, nl, tid_l, rb, 0);
      STAMP(4);
      if (A.stats != nullptr && tid == 0) {
        unsigned long long edges = 0;
        for (int a = 0; a < rb; ++a) edges += (unsigned long long)sm.cntrow[r0 + a];
        atomicAdd(&A.stats[0], (unsigned long long)sm.npairs);
        atomicAdd(&A.stats[1], edges);
      }
      constexpr int NT = H / 32;
      // the hand-off granules of layer k's tail: {value, tag(k)} in parity k & 1
      auto put = [&](int k, int a, int c, float v) {   // a: row within the block, c: 0..2 pos, 3.. h
        const uint64_t g = ((uint64_t)xtag(epoch, k) << 32) | (uint64_t)__float_as_uint(v);
        __hip_atomic_store(xmine + (k & 1) * XSLOT + a * XG + c, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      };
      auto get = [&](int k, int a, int c) {            // a: row within the partner's block
        const uint64_t g = fs_poll(F, xpart + (k & 1) * XSLOT + a * XG + c, xtag(epoch, k), X.spin_limit);
        return __uint_as_float((uint32_t)g);
      };
      const float* nb = F.nb[it & 1];
      // the partner's features from the previous layer's tail, published there a
      // pair build ago (needed from the first GEMM0 on: fs_edge_tiles' first barrier
      // orders these writes before it)
      static_assert(HALF * NFMAX <= BLOCK, "one partner feature granule per thread");
      if (hget) {
        const int a = he / nfl, q = he - a * nfl;
        sm.h[(pr0 + a) * NFP + q] = ((uint32_t)(hg >> 32) == xtag(epoch, it - 1) && X.spin_limit > 0)
                                        ? __uint_as_float((uint32_t)hg) : get(it - 1, a, 3 + q);
      }
      fs_edge_tiles<H, KS0>(F, Lp, L, Ml, nfl, tid_l, r0, rb, Wt, nb STAMP_PASS);
      STAMP(5);
      // ---- tail T1: node_nn items on waves 0 .. NT - 1; on the others the
      // velocity / position update of the workgroup's rows (dynamics.py:15-20
      // forward, 33-35 + the next half-step 29 in reverse: Q from the tiles' first
      // step, the forces from the tiles), the positions published at once; the
      // next layer's bias images requested
      FsBias nbias{0.f, 0.f};
      if (more) nbias = fs_bias_load<H>(Lpn, L, tid_l);
      constexpr int GT = NT * 64;   // threads per wave group
      if (w < NT) {
        fs_node_g(F, Lp, L, tid_l, r0, rb, nfl, nb STAMP_PASS);
      } else {
        for (int a = tid_l - GT; a < rb; a += BLOCK - GT) {
          const int ag = r0 + a;
          float q = 0.f;
#pragma unroll
          for (int tp = 0; tp < NT; ++tp) q += sm.u.nd.qp[tp][a];
          q += nb[3 * H + NFMAX];
          const float eq = expf(q);
          const float inv = 1.f / fmaxf((float)sm.cntrow[ag], 1.f);   // helpers.py:63-70
          for (int d = 0; d < 3; ++d) {
            const float Fd = sm.agg[a * AST + H + d] * inv * A.cw;
            float v, p = sm.pos[ag * 3 + d];
            if (!REV) {
              v = eq * sm.vel[ag * 3 + d] + Fd * A.dt;
              p = pbc1(p + v * A.dt, pbox(ag, d));
            } else {
              v = (sm.vel[ag * 3 + d] - Fd * A.dt) / eq;
              if (more) p = pbc1(p - v * A.dt, pbox(ag, d));
            }
            sm.vel[ag * 3 + d] = v;
            sm.pos[ag * 3 + d] = p;
            if (SPLIT == 2 && more) put(it, a, d, p);
          }
          if (!REV) ldj += q;
        }
        // the partner's positions, published in its own T1: polled here, behind
        // the node_nn items of this T1
        if (SPLIT == 2 && more)
          for (int e = tid_l - GT; e < prb * 3; e += BLOCK - GT) {
            const int a = e / 3, d = e - a * 3;
            sm.pos[(pr0 + a) * 3 + d] = get(it, a, d);
          }
      }
      __syncthreads();
      STAMP(6);
      // ---- tail T2: the features' update (G), published
      if (tid == 0) {
        if (small_operands(sm.big)) sm.err |= ENFLOW_ERR_SMALL;
        sm.big = 0u;
      }
      if (w < NT) {   // dynamics.py:21-22 (forward) / 32 + the next half-step 28 (reverse)
        for (int e = tid_l; e < rb * nfl; e += GT) {
          const int a = e / nfl, q = e - a * nfl, ag = r0 + a;
          float G = 0.f;
#pragma unroll
          for (int tp = 0; tp < NT; ++tp) G += sm.u.nd.gp[tp][q][a];
          G += nb[3 * H + q];
          const float gn = REV ? sm.g[ag * NFP + q] - G * A.dt : sm.g[ag * NFP + q] + G * A.dt;
          sm.g[ag * NFP + q] = gn;
          float hv = sm.h[ag * NFP + q];
          if (!REV) hv += gn * A.dt;
          else if (more) hv -= gn * A.dt;
          sm.h[ag * NFP + q] = hv;
          if (SPLIT == 2 && more) put(it, a, 3 + q, hv);
        }
      }
      if (more) fs_bias_store(F, Lpn, L, tid_l, nbias, (it + 1) & 1);
      __syncthreads();
      STAMP(7);
    }

    if (REV) {   // dequantize.reverse (argmax.py:27-28 / floor.py:13), the workgroup's atoms
      for (int a = r0 + tid; a < r0 + rb; a += BLOCK) {
        if (A.dequant_kind == ENFLOW_DEQUANT_ARGMAX) {
          int best = 0;
          float bv = sm.h[a * NFP];
          for (int q = 1; q < nf; ++q)
            if (sm.h[a * NFP + q] > bv) { bv = sm.h[a * NFP + q]; best = q; }
          A.argmax_idx[M.a0 + a] = best;
          atomicMax(A.max_idx, best);
        } else if (A.dequant_kind == ENFLOW_DEQUANT_FLOOR) {
          for (int q = 0; q < nf; ++q) sm.h[a * NFP + q] = floorf(sm.h[a * NFP + q]);
        }
      }
      __syncthreads();
    }
    bool bad = false;
    for (int e = tid; e < rb * 3; e += BLOCK) {
      const int ee = r0 * 3 + e;
      const float p = sm.pos[ee], v = sm.vel[ee];
      A.pos[(size_t)M.a0 * 3 + ee] = p;
      A.vel[(size_t)M.a0 * 3 + ee] = v;
      bad |= !__builtin_isfinite(p) || !__builtin_isfinite(v);
    }
    for (int e = tid; e < rb * nf; e += BLOCK) {
      const int a = r0 + e / nf, q = e % nf;
      const float hv = sm.h[a * NFP + q], gv = sm.g[a * NFP + q];
      A.h[(size_t)(M.a0 + a) * nf + q] = hv;
      A.g[(size_t)(M.a0 + a) * nf + q] = gv;
      bad |= (!REV && !__builtin_isfinite(hv)) || !__builtin_isfinite(gv);
    }
    if (bad) atomicOr(&sm.err, ENFLOW_ERR_RANGE);
    __syncthreads();
    if (tid == 0) {
      int err = sm.err;
      if (F.timeout) err |= ENFLOW_ERR_HANDOFF;
      if (err) {
        atomicOr(A.err, err);
        if (A.mol_err) atomicOr(&A.mol_err[m], err);
      }
    }
  }
  STAMP(19);
  STAMP_FLUSH
  if (REV) return;
  // log|detJ|: this workgroup's partial, then the last workgroup to finish sums
  // them in a fixed order (per molecule half 0 + half 1, then
  // reduce_ldj_kernel's strided double sums and tree) and resets the ticket.
  // The partials are sc1 stores drained before the ticket add, and read with sc1
  // loads by the workgroup whose add came last (MI355X_MICROARCH.md, hand-off
  // table row 1): no cache-wide fence.
  const float s = block_sum(sm, ldj);
  __shared__ int last;
  if (tid == 0) {
    if (s != s || !__builtin_isfinite(s)) {
      if (active) {
        atomicOr(A.err, ENFLOW_ERR_RANGE);
        if (A.mol_err) atomicOr(&A.mol_err[m], ENFLOW_ERR_RANGE);
      }
    }
    __hip_atomic_store(&X.part[b], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(&X.ctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)X.blocks - 1;
  }
  __syncthreads();
  if (!last) return;
  constexpr int RT = 256;
  double* red = reinterpret_cast<double*>(sm.agg);
  double acc = 0.0;
  if (tid < RT)
    for (int mm = tid; mm < A.num_mols; mm += RT) {
      float v;
      if (SPLIT == 2) {
        const int b0 = (mm >> 3) * 16 + (mm & 7);
        v = __hip_atomic_load(&X.part[b0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
            __hip_atomic_load(&X.part[b0 + 8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        v = __hip_atomic_load(&X.part[mm], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      A.ldj_mol[mm] = v;
      acc += (double)v;
    }
  if (tid < RT) red[tid] = acc;
  __syncthreads();
  for (int off = RT / 2; off > 0; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  if (tid == 0) {
    A.ldj_total[0] = (float)(red[0] + A.ldj_cst);
    __hip_atomic_store(&X.ctl[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&X.ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// reverse launches have no ticket: the epoch advances in a one-thread kernel
// after them (stream order) so the next launch's tags differ
__global__ void fs_epoch_kernel(uint32_t* ctl) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(&ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace enflow_fs

// ---------------------------------------------------------------------------
// host side: per-(device, stream) hand-off buffers (allocated on first use,
// deliberately never freed: a static destructor running after the HIP runtime
// has torn down must not call into it), the instance choice
// ---------------------------------------------------------------------------
namespace {
struct XBuf {
  int dev;
  hipStream_t st;
  int cap;            // molecules
  uint64_t* xch;
  uint32_t* ctl;
  float* part;
};
std::mutex g_mu;
XBuf g_buf[64];
int g_nbuf = 0;
int g_split_threshold = -1;   // SPLIT = 2 for batches of at most this many molecules (-1: CUs / 2)
int g_fs_threshold = -1;      // SPLIT = 1 for batches of at most this many molecules (-1: CUs; 0: off)
constexpr int kSpinDefault = 1 << 20;
int g_spin_limit = kSpinDefault;   // polls per hand-off wait (enflow_set_handoff_spin_limit)
int g_cus[64];

int cus_of(int dev) {
  if (dev < 0 || dev >= 64) return 0;
  if (g_cus[dev] == 0) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) return 0;
    g_cus[dev] = c;
  }
  return g_cus[dev];
}

XBuf* buffers(int dev, hipStream_t st, int mols) {
  std::lock_guard<std::mutex> lk(g_mu);
  XBuf* hit = nullptr;
  for (int i = 0; i < g_nbuf; ++i)
    if (g_buf[i].dev == dev && g_buf[i].st == st) hit = &g_buf[i];
  if (hit && hit->cap >= mols) return hit;
  if (!hit) {
    if (g_nbuf >= 64) return nullptr;
    hit = &g_buf[g_nbuf++];
    hit->dev = dev;
    hit->st = st;
    hit->cap = 0;
    hit->ctl = nullptr;
  }
  // (re)size: the old buffers may still be read by queued launches -- leaked
  const int cap = mols < 128 ? 128 : mols;
  const size_t blocks = (size_t)2 * cap + 16;
  uint64_t* x = nullptr;
  float* p = nullptr;
  if (hipMalloc(&x, sizeof(uint64_t) * (size_t)cap * 4 * enflow_fs::XSLOT) != hipSuccess) return nullptr;
  if (hipMalloc(&p, sizeof(float) * blocks) != hipSuccess) return nullptr;
  if (hipMemsetAsync(x, 0, sizeof(uint64_t) * (size_t)cap * 4 * enflow_fs::XSLOT, st) != hipSuccess) return nullptr;
  if (!hit->ctl) {
    uint32_t* c = nullptr;
    if (hipMalloc(&c, sizeof(uint32_t) * 4) != hipSuccess) return nullptr;
    if (hipMemsetAsync(c, 0, sizeof(uint32_t) * 4, st) != hipSuccess) return nullptr;
    hit->ctl = c;
  }
  hit->xch = x;
  hit->part = p;
  hit->cap = cap;
  return hit;
}
}  // namespace

int enflow_fs_split_for(int num_mols) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const int cus = cus_of(dev);
  const int t2 = g_split_threshold >= 0 ? g_split_threshold : cus / 2;
  if (num_mols > 0 && num_mols <= t2 && 2 * num_mols <= cus) return 2;
  const int t1 = g_fs_threshold >= 0 ? g_fs_threshold : cus;   // one workgroup per molecule and CU
  if (num_mols > 0 && num_mols <= t1) return 1;
  return 0;
}

bool enflow_fs_launch(int H, bool rev, int prec, int num_mols, hipStream_t st, const void* flow_args) {
  const auto& A = *static_cast<const enflow_fs::FlowArgs*>(flow_args);
  if (H != 128 || prec != ENFLOW_PREC_F16X3 || A.tape != nullptr || A.nf > NFMAX || A.mol_list != nullptr ||
      A.n_layers < 1)
    return false;
  int split = enflow_fs_split_for(num_mols);
  if (split == 0) return false;
  // in place, a half could overwrite rows its partner has not read yet (a
  // one-layer flow has no hand-off to order them), and a re-run after
  // ENFLOW_ERR_HANDOFF would start from overwritten inputs: one workgroup per
  // molecule instead (it reads its whole molecule before it writes anything)
  if (split == 2 && !(A.h_in && A.g_in && A.pos_in && A.vel_in)) split = 1;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  XBuf* B = buffers(dev, st, num_mols);
  if (!B) return false;
  enflow_fs::FsArgs X;
  X.xch = B->xch;
  X.ctl = B->ctl;
  X.part = B->part;
  X.split = split;
  X.blocks = split == 2 ? ((2 * num_mols + 15) / 16) * 16 : num_mols;
  X.spin_limit = g_spin_limit;
  enflow_fs::FlowArgs Ak = A;
  Ak.ticket = nullptr;   // the instance reduces through its own ticket (FsArgs::ctl)
  Ak.num_mols = num_mols;   // (the reverse entry leaves it unset: whole-tile kernels index by block)
  const char* name = rev ? "lf_fs_kernel<rev>" : "lf_fs_kernel<fwd>";
  const dim3 grid(X.blocks), blk(BLOCK);
#define FS_GO(RV, SP, K0) ENFLOW_TIMED(name, st, hipLaunchKernelGGL((enflow_fs::lf_fs_kernel<128, RV, SP, K0>), grid, blk, 0, st, Ak, X))
  const bool k1 = enflow_fs::gemm0_ksteps(A.nf) == 1;   // nf <= 7 (radial in slot 7): one edge_nn.0 k-slice
  if (split == 2) {
    if (rev) { if (k1) FS_GO(true, 2, 1); else FS_GO(true, 2, KS0MAX); }
    else { if (k1) FS_GO(false, 2, 1); else FS_GO(false, 2, KS0MAX); }
  } else {
    if (rev) { if (k1) FS_GO(true, 1, 1); else FS_GO(true, 1, KS0MAX); }
    else { if (k1) FS_GO(false, 1, 1); else FS_GO(false, 1, KS0MAX); }
  }
#undef FS_GO
  if (rev && split == 2) hipLaunchKernelGGL(enflow_fs::fs_epoch_kernel, dim3(1), dim3(64), 0, st, B->ctl);
  return true;
}

extern "C" {
#ifdef ENFLOW_STAMPS
// diagnostic build only: this TU's stamp accumulators
int enflow_read_stamps_fs(unsigned long long* host_out, int reset) {
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(enflow_fs::enflow_stamp_acc), sizeof(unsigned long long) * NSTAMP) !=
      hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[NSTAMP] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(enflow_fs::enflow_stamp_acc), z, sizeof(z)) != hipSuccess) return -1;
  }
  return NSTAMP;
}
#endif
int enflow_set_split_threshold(int max_mols) {
  const int prev = g_split_threshold;
  g_split_threshold = max_mols < 0 ? -1 : max_mols;
  return prev;
}
int enflow_set_fs_threshold(int max_mols) {
  const int prev = g_fs_threshold;
  g_fs_threshold = max_mols < 0 ? -1 : max_mols;
  return prev;
}
int enflow_set_handoff_spin_limit(int polls) {
  const int prev = g_spin_limit;
  g_spin_limit = polls < 0 ? kSpinDefault : polls;
  return prev;
}
}  // extern "C"
