// enflow_large.hip -- the coupling flow for molecules / periodic systems larger
// than the fused kernel's LDS image (> 256 atoms; e.g. the reference's
// example/generate.yaml: one 2944-atom Lennard-Jones box, batch 1).
//
// The fused kernel (enflow_flow.hip) keeps a whole molecule in one
// workgroup's LDS across all layers.  A large system does not fit, and every
// layer's neighbour list depends on the previous layer's positions, so here
// each layer is a short sequence of grid-wide launches on one stream:
//
//   lg_images_kernel   one thread per atom: (reverse only) the pre-network
//                      half step h -= g dt, pos = pbc(pos - vel dt)
//                      (dynamics.py:28-30), then the 27-bit periodic-image
//                      mask (helpers.py:10-27)
//   lg_idmap_kernel    one workgroup per molecule: id_mapping[q] for q < n,
//                      the q-th surviving image in (image, atom) order
//                      (helpers.py:25-27), 27 block scans of the mask bits
//   lg_pairs_kernel    one wave per row atom i: for every column q the number
//                      of i's images within r_cut of atom q, labelled
//                      id_mapping[q] (base.py:133-139: both hit columns are
//                      mapped through id_mapping, self labels dropped); the
//                      nonzero counts are written as (label, multiplicity)
//                      words in q order into row i's slot of the pair buffer
//                      (row stride max_mol_atoms: a row has at most n words),
//                      plus the row's edge count (the segment-mean divisor)
//   lg_layer_kernel    one workgroup per 32-row block: the rows' h / pos in
//                      the LDS image, the rows' pair words streamed through
//                      the LDS pair buffer in passes of PC, the same MFMA edge
//                      tiles / segment sums / node phase as the fused kernel
//                      (edge_tiles<..., BIG = true>: column atoms read from
//                      global memory, L2-resident), then the leapfrog update
//                      of the rows.  Forward: pos / h of the next layer go to
//                      a second buffer (other blocks still read this layer's),
//                      vel / g in place; log|detJ| per block accumulated in
//                      fixed layer order.  Reverse: g / vel in place.
//
// Neighbour search is the reference's own all-pairs-over-27-images test
// (O(27 n^2) per layer, as Data.edges); per-row work is wave-uniform.  All
// reductions run in a fixed order: results are bitwise reproducible.
#include <stdlib.h>

#include "enflow_large.h"

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// row blocks of rbl atoms per molecule: blk_start[m] = sum_{m' < m} ceil(n_m' / rbl)
__global__ void __launch_bounds__(BLOCK) lg_setup_kernel(const int32_t* __restrict__ mol_ptr, int num_mols, int rbl,
                                                         int32_t* __restrict__ blk_start) {
  __shared__ int part[BLOCK];
  const int tid = threadIdx.x;
  const int per = (num_mols + BLOCK - 1) / BLOCK;
  const int m0 = min(num_mols, tid * per), m1 = min(num_mols, m0 + per);
  int s = 0;
  for (int m = m0; m < m1; ++m) s += (mol_ptr[m + 1] - mol_ptr[m] + rbl - 1) / rbl;
  part[tid] = s;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int k = 0; k < BLOCK; ++k) { const int v = part[k]; part[k] = acc; acc += v; }
    blk_start[num_mols] = acc;
  }
  __syncthreads();
  int acc = part[tid];
  for (int m = m0; m < m1; ++m) {
    blk_start[m] = acc;
    acc += (mol_ptr[m + 1] - mol_ptr[m] + rbl - 1) / rbl;
  }
}

__global__ void __launch_bounds__(BLOCK) lg_images_kernel(LgArgs B, int rev) {
  const int a = blockIdx.x * BLOCK + threadIdx.x;
  if (a >= B.num_atoms) return;
  const int m = seg_of(B.mol_ptr, B.num_mols, a);
  const int a0 = B.mol_ptr[m], nf = B.nf;
  float p[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) p[d] = B.pos[(size_t)a * 3 + d];
  if (rev) {   // dynamics.py:28-30
    for (int q = 0; q < nf; ++q) B.h[(size_t)a * nf + q] -= B.g[(size_t)a * nf + q] * B.dt;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      p[d] = pbc1(p[d] - B.vel[(size_t)a * 3 + d] * B.dt, B.box[(size_t)a * 3 + d]);
      B.pos[(size_t)a * 3 + d] = p[d];
    }
  }
  // the molecule's edge box is its first atom's (base.py:130)
  const float bx = B.box[(size_t)a0 * 3 + 0], by = B.box[(size_t)a0 * 3 + 1], bz = B.box[(size_t)a0 * 3 + 2];
  const float rc = B.r_cut[m];
  const float rx = bx + rc, ry = by + rc, rz = bz + rc;   // helpers.py:20
  uint32_t mk = 0u;
  for (int s = 0; s < 27; ++s) {
    const float sx = (p[0] + shift_of(s % 3, bx)) / rx;
    const float sy = (p[1] + shift_of((s / 3) % 3, by)) / ry;
    const float sz = (p[2] + shift_of(s / 9, bz)) / rz;
    if (sx * sx + sy * sy + sz * sz <= 1.0f) mk |= 1u << s;
  }
  B.mask[a] = mk;
}

// id_mapping[q], q < n: the q-th surviving (image, atom) in image-major order.
// Each thread counts the 27 image bits over its contiguous atom chunk, one
// block scan of the 27 counts gives every (image, chunk) its output offset.
constexpr int IDB = 256, IDW = IDB / 64;   // lg_idmap_kernel: 4 waves per molecule (~200 VGPRs)
__global__ void __launch_bounds__(IDB) lg_idmap_kernel(LgArgs B) {
  constexpr int MK_LDS = 12288;   // masks of molecules up to this size staged in LDS
  __shared__ uint32_t mk_l[MK_LDS];
  __shared__ int wsum[27][IDW];
  const int m = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int a0 = B.mol_ptr[m], n = B.mol_ptr[m + 1] - a0;
  const int per = (n + IDB - 1) / IDB;
  const int c0 = min(n, tid * per), c1 = min(n, c0 + per);
  const uint32_t* mk = n <= MK_LDS ? mk_l : B.mask + a0;
  int32_t* idm = B.idmap + a0;
  __shared__ float red[6][IDW];
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int a = tid; a < n; a += IDB) {
    idm[a] = -1;
    if (n <= MK_LDS) mk_l[a] = B.mask[a0 + a];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const float x = B.pos[(size_t)(a0 + a) * 3 + d];
      lo[d] = fminf(lo[d], x);
      hi[d] = fmaxf(hi[d], x);
    }
  }
  // the molecule's bounding box (min / max: order-independent), for the pair
  // search's image culling
#pragma unroll
  for (int d = 0; d < 3; ++d) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo[d] = fminf(lo[d], __shfl_xor(lo[d], o, 64));
      hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], o, 64));
    }
    if (lane == 0) { red[d][w] = lo[d]; red[3 + d][w] = hi[d]; }
  }
  __syncthreads();
  if (tid < 6) {
    float v = red[tid][0];
    for (int k = 1; k < IDW; ++k) v = tid < 3 ? fminf(v, red[tid][k]) : fmaxf(v, red[tid][k]);
    B.aabb[(size_t)m * 6 + tid] = v;
  }
  // the thread's chunk of masks in registers (molecules up to IDB * MR atoms)
  constexpr int MR = 16;
  const bool regs = per <= MR;
  uint32_t mr[MR];
#pragma unroll
  for (int k = 0; k < MR; ++k) mr[k] = (regs && c0 + k < c1) ? mk[c0 + k] : 0u;
  int cnt[27];
#pragma unroll
  for (int s = 0; s < 27; ++s) cnt[s] = 0;
  if (regs) {
#pragma unroll
    for (int k = 0; k < MR; ++k)
#pragma unroll
      for (int s = 0; s < 27; ++s) cnt[s] += (mr[k] >> s) & 1u;
  } else {
    for (int a = c0; a < c1; ++a) {
      const uint32_t v = mk[a];
#pragma unroll
      for (int s = 0; s < 27; ++s) cnt[s] += (v >> s) & 1u;
    }
  }
  int base[27];
#pragma unroll
  for (int s = 0; s < 27; ++s) {
    const int incl = wave_incl_scan(cnt[s]);
    base[s] = incl - cnt[s];
    if (lane == 63) wsum[s][w] = incl;
  }
  __syncthreads();
  int prefix = 0;   // surviving images of the earlier image indices
#pragma unroll
  for (int s = 0; s < 27; ++s) {
    int tot = 0, before = 0;
    for (int k = 0; k < IDW; ++k) {
      if (k < w) before += wsum[s][k];
      tot += wsum[s][k];
    }
    base[s] += prefix + before;
    prefix += tot;
  }
  // prefix < n: columns q >= prefix keep id_mapping -1 (initialised above); the
  // reference raises only if such a column has a hit (lg_pairs_kernel)
#pragma unroll
  for (int s = 0; s < 27; ++s) {   // unrolled: cnt / base stay in registers
    int o = base[s];
    if (o < n) {
      if (regs) {
#pragma unroll
        for (int k = 0; k < MR; ++k)
          if (((mr[k] >> s) & 1u) && o < n) idm[o++] = c0 + k;   // mr[k] = 0 past the chunk
      } else {
        for (int a = c0; a < c1 && o < n; ++a)
          if ((mk[a] >> s) & 1u) idm[o++] = a;
      }
    }
  }
}

// pair words of the rows of one row block: (id_mapping[q] << 5) | (multiplicity
// << 27), q order; column positions / labels staged in LDS in chunks of QC
// atoms shared by the block's waves (one wave per row)
__global__ void __launch_bounds__(BLOCK) lg_pairs_kernel(LgArgs B) {
  constexpr int QC = 1024;
  __shared__ float qp[QC * 3];
  __shared__ int qid[QC];
  __shared__ float img[WAVES][27 * 3];   // the current row's surviving images (per wave)
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x, tid = threadIdx.x;
  if (b >= B.blk_start[B.num_mols]) return;
  const int m = seg_of(B.blk_start, B.num_mols, b);
  const int a0 = B.mol_ptr[m], n = B.mol_ptr[m + 1] - a0;
  const int r0 = (b - B.blk_start[m]) * B.rbl, rb = min(B.rbl, n - r0);
  const float bx = B.box[(size_t)a0 * 3 + 0], by = B.box[(size_t)a0 * 3 + 1], bz = B.box[(size_t)a0 * 3 + 2];
  const float rc = B.r_cut[m], r_sq = rc * rc;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  float bb[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) bb[k] = B.aabb[(size_t)m * 6 + k];
  constexpr int RPW = 8;   // rows per wave (rbl <= 32)
  int np[RPW], edges[RPW];
#pragma unroll
  for (int k = 0; k < RPW; ++k) np[k] = edges[k] = 0;
  for (int q0 = 0; q0 < n; q0 += QC) {
    const int qn = min(QC, n - q0);
    __syncthreads();   // previous chunk consumed
    for (int e = tid; e < qn * 3; e += BLOCK) qp[e] = B.pos[(size_t)(a0 + q0) * 3 + e];
    for (int e = tid; e < qn; e += BLOCK) qid[e] = B.idmap[a0 + q0 + e];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const int il = w + WAVES * k;
      if (il >= rb) break;   // wave-uniform
      const int a = a0 + r0 + il;
      const uint32_t mk = B.mask[a];
      // image list of the row (wave-private LDS): the surviving images that
      // can reach the molecule's bounding box at all (farther than r_cut from
      // it, with a 1e-4 relative margin over fp32 rounding, no atom can hit)
      uint32_t cand = 0u;
      float ix = 0.f, iy = 0.f, iz = 0.f;
      if (lane < 27 && ((mk >> lane) & 1u)) {
        const int s = lane;
        ix = B.pos[(size_t)a * 3 + 0] + shift_of(s % 3, bx);
        iy = B.pos[(size_t)a * 3 + 1] + shift_of((s / 3) % 3, by);
        iz = B.pos[(size_t)a * 3 + 2] + shift_of(s / 9, bz);
        const float ex = fmaxf(fmaxf(bb[0] - ix, ix - bb[3]), 0.f);
        const float ey = fmaxf(fmaxf(bb[1] - iy, iy - bb[4]), 0.f);
        const float ez = fmaxf(fmaxf(bb[2] - iz, iz - bb[5]), 0.f);
        cand = (ex * ex + ey * ey + ez * ez) <= r_sq * 1.0001f ? 1u : 0u;
      }
      const uint64_t cb = __ballot(cand != 0u);
      const int ni = __popcll(cb);
      if (cand) {
        const int slot = __popcll(cb & lt);
        img[w][slot * 3 + 0] = ix;
        img[w][slot * 3 + 1] = iy;
        img[w][slot * 3 + 2] = iz;
      }
      wave_lds_sync();
      uint32_t* out = B.pairs + (size_t)a * B.max_n;
      for (int qc = 0; qc < qn; qc += 64) {
        const int ql = qc + lane;
        int c = 0, jl = -1;
        if (ql < qn) {
          jl = qid[ql];
          if (jl != r0 + il) {   // self pair by label (base.py:139)
            const float qx = qp[ql * 3 + 0], qy = qp[ql * 3 + 1], qz = qp[ql * 3 + 2];
            for (int t = 0; t < ni; ++t) {   // wave-uniform trip count, broadcast LDS reads
              const float dx = img[w][t * 3 + 0] - qx, dy = img[w][t * 3 + 1] - qy, dz = img[w][t * 3 + 2] - qz;
              c += (dx * dx + dy * dy + dz * dz < r_sq) ? 1 : 0;
            }
            if (jl < 0 && c > 0) {   // a hit on column q past id_mapping: the reference's IndexError
              atomicOr(B.err, ENFLOW_ERR_FEW_IMAGES);
              c = 0;
            }
          }
        }
        const uint64_t bal = __ballot(c > 0);
        if (c > 0) out[np[k] + __popcll(bal & lt)] = ((uint32_t)jl << 5) | ((uint32_t)c << 27);
        if (B.smap && ql < qn)   // training backward: column q's slot in the row (dense, coalesced)
          B.smap[(size_t)a * B.max_n + q0 + ql] = c > 0 ? np[k] + __popcll(bal & lt) : -1;
        np[k] += __popcll(bal);
        edges[k] += c;
      }
      wave_lds_sync();   // image list reused by the wave's next row
    }
  }
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int il = w + WAVES * k;
    if (il >= rb) break;
    const int e = wave_sum_i(edges[k]);
    if (lane == 0) {
      B.npairs[a0 + r0 + il] = np[k];
      B.cntrow[a0 + r0 + il] = e;
    }
  }
}

// one EGCL layer (+ leapfrog update) for one 32-row block.  mode 0: flow
// forward, 1: flow reverse, 2: EGCL only (Q, F, G to Qo / Fo / Go).
template <int H, int PREC, bool VAR>
__global__ void __launch_bounds__(BLOCK, 1) lg_layer_kernel(LgArgs B, int mode) {
  using S = Smem<H, 32, 32>;
  __shared__ S sm;
  __shared__ int roff[33];
  constexpr int AST = S::AST;
  constexpr int PC = S::PC;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (b >= B.blk_start[B.num_mols]) return;
  const int m = seg_of(B.blk_start, B.num_mols, b);
  MolRef M;
  M.a0 = B.mol_ptr[m];
  M.n = B.mol_ptr[m + 1] - M.a0;
  M.rc = B.r_cut[m];
  M.bx = B.box[(size_t)M.a0 * 3 + 0];
  M.by = B.box[(size_t)M.a0 * 3 + 1];
  M.bz = B.box[(size_t)M.a0 * 3 + 2];
  const int r0 = (b - B.blk_start[m]) * B.rbl, rb = min(B.rbl, M.n - r0);
  const int g0 = M.a0 + r0;   // first row atom (global)
  STAMP_DECL   // diagnostic builds only (-DENFLOW_STAMPS)
  const int nf = B.nf;
  const EgclLayout L = egcl_layout(H, nf);
  for (int e = tid; e < rb * 3; e += BLOCK) sm.pos[e] = B.pos[(size_t)g0 * 3 + e];
  for (int e = tid; e < 32 * NFP; e += BLOCK) {   // rows zero-padded past nf and rb
    const int a = e / NFP, q = e - a * NFP;
    sm.h[e] = (a < rb && q < nf) ? B.h[(size_t)(g0 + a) * nf + q] : 0.f;
  }
  if (tid < 32) sm.cntrow[tid] = tid < rb ? B.cntrow[g0 + tid] : 0;
  if (tid == 0) {
    sm.err = 0;
    sm.big = 0u;
    int acc = 0;
    for (int a = 0; a < rb; ++a) { roff[a] = acc; acc += B.npairs[g0 + a]; }
    for (int a = rb; a <= 32; ++a) roff[a] = acc;
  }
  __syncthreads();
  const int tot = roff[32];
  const float* cpos = B.pos + (size_t)M.a0 * 3;
  const float* ch = B.h + (size_t)M.a0 * nf;
  for (int p0 = 0;;) {   // at least one pass (zeroes the aggregates)
    const int cnt = min(PC, tot - p0);
    for (int e = tid; e < cnt; e += BLOCK) {
      const int pe = p0 + e;
      int lo = 0, hi = rb;   // row il: roff[il] <= pe < roff[il + 1]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (roff[mid] <= pe) lo = mid;
        else hi = mid;
      }
      sm.pairs[e] = B.pairs[(size_t)(g0 + lo) * B.max_n + (pe - roff[lo])] | (uint32_t)lo;
    }
    if (tid == 0) sm.npairs = max(cnt, 0);
    __syncthreads();
    edge_tiles<H, 32, 32, PREC, VAR, true>(sm, B.layer, L, M, nf, tid, 0, rb, p0 == 0 STAMP_PASS, cpos, ch);
    p0 += PC;
    if (p0 >= tot) break;
  }
  if constexpr (PREC != PREC_F32) node_phase_x3<H, 32, 32, VAR>(sm, B.layer, L, rb, nf, tid, 0, rb);
  else node_phase<H, 32, 32, VAR>(sm, B.layer, L, rb, nf, tid, 0, rb);
  if constexpr (PREC == PREC_F16X3) {   // small-operand guard of the row block (BIGK_*)
    if (tid == 0 && small_operands(sm.big)) sm.err |= ENFLOW_ERR_SMALL;
  }
  if (tid == 0 && sm.err) atomicOr(B.err, sm.err);   // edge tiles' range check (split precision)

  const bool tape = mode == 0 && B.tape != nullptr;
  if (tape) {   // training tape (as the fused kernel's): layer-input h / pos, message sums, Q
    const TapeLayout T = tape_layout(B.num_atoms, nf, H, B.n_layers);
    const size_t la = (size_t)B.layer_idx * B.num_atoms + g0;
    float* hx = B.tape + T.hx + la * T.ldhx;
    for (int e = tid; e < rb * T.ldhx; e += BLOCK) {
      const int a = e / T.ldhx, c = e - a * T.ldhx;
      hx[e] = c < nf ? sm.h[a * NFP + c] : sm.agg[a * AST + (c - nf)];
    }
    for (int e = tid; e < rb * 3; e += BLOCK) B.tape[T.pos + la * 3 + e] = sm.pos[e];
    for (int a = tid; a < rb; a += BLOCK) B.tape[T.q + la + a] = sm.Q[a];
    if (tid == 0) atomicAdd(B.pair_rows + B.layer_idx, (tot + 31) & ~31);   // the backward's pair rows
  }
  float ldj = 0.f;
  for (int a = tid; a < rb; a += BLOCK) {
    const size_t ga = (size_t)(g0 + a);
    if (tape) {   // layer-input g / vel, read before the update below overwrites them (same thread)
      const TapeLayout T = tape_layout(B.num_atoms, nf, H, B.n_layers);
      const size_t la = (size_t)B.layer_idx * B.num_atoms + ga;
      for (int qf = 0; qf < nf; ++qf) B.tape[T.g + la * nf + qf] = B.g[ga * nf + qf];
      for (int d = 0; d < 3; ++d) B.tape[T.vel + la * 3 + d] = B.vel[ga * 3 + d];
    }
    const float q = sm.Q[a];
    const float inv = 1.f / fmaxf((float)sm.cntrow[a], 1.f);   // helpers.py:63-70
    float F[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) F[d] = sm.agg[a * AST + H + d] * inv * B.cw;
    if constexpr (PREC != PREC_F32) {   // split-precision GEMM out of range (ENFLOW_ERR_RANGE)
      bool bad = !__builtin_isfinite(q) || !__builtin_isfinite(F[0]) || !__builtin_isfinite(F[1]) ||
                 !__builtin_isfinite(F[2]);
      for (int qf = 0; qf < nf; ++qf) bad |= !__builtin_isfinite(sm.G[a * NFP + qf]);
      if (bad) atomicOr(B.err, ENFLOW_ERR_RANGE);
    }
    if (mode == 2) {   // EGCL.forward outputs
      B.Qo[ga] = q;
      for (int d = 0; d < 3; ++d) B.Fo[ga * 3 + d] = F[d];
      for (int qf = 0; qf < nf; ++qf) B.Go[ga * nf + qf] = sm.G[a * NFP + qf];
    } else if (mode == 0) {   // dynamics.py:15-22
      const float eq = expf(q);
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const float v = eq * B.vel[ga * 3 + d] + F[d] * B.dt;
        B.vel[ga * 3 + d] = v;
        B.pos2[ga * 3 + d] = pbc1(sm.pos[a * 3 + d] + v * B.dt, B.box[ga * 3 + d]);
      }
      for (int qf = 0; qf < nf; ++qf) {
        const float gn = B.g[ga * nf + qf] + sm.G[a * NFP + qf] * B.dt;
        B.g[ga * nf + qf] = gn;
        B.h2[ga * nf + qf] = sm.h[a * NFP + qf] + gn * B.dt;
      }
      ldj += q;
    } else {   // dynamics.py:32-35
      const float eq = expf(q);
      for (int qf = 0; qf < nf; ++qf) B.g[ga * nf + qf] -= sm.G[a * NFP + qf] * B.dt;
#pragma unroll
      for (int d = 0; d < 3; ++d) B.vel[ga * 3 + d] = (B.vel[ga * 3 + d] - F[d] * B.dt) / eq;
    }
  }
  if (mode == 0) {
    const float s = block_sum(sm, ldj);
    if (tid == 0) B.ldj_blk[b] += s;   // fixed layer order: one writer per block and launch
  }
}

// dequantize (forward) per row block: ArgMax.forward (argmax.py:13-25) on the
// rows, or Floor (floor.py:8-10); initialises ldj_blk
template <int H>
__global__ void __launch_bounds__(BLOCK) lg_dequant_kernel(LgArgs B, int kind, const float* __restrict__ dq,
                                                           const float* __restrict__ noise, float scale) {
  using S = Smem<H, 32, 32>;
  __shared__ S sm;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (b >= B.blk_start[B.num_mols]) return;
  const int m = seg_of(B.blk_start, B.num_mols, b);
  const int a0 = B.mol_ptr[m], n = B.mol_ptr[m + 1] - a0;
  const int r0 = (b - B.blk_start[m]) * B.rbl, rb = min(B.rbl, n - r0);
  const int g0 = a0 + r0, nf = B.nf;
  float lq = 0.f;
  if (kind == ENFLOW_DEQUANT_ARGMAX) {
    for (int e = tid; e < 32 * NFP; e += BLOCK) {
      const int a = e / NFP, q = e - a * NFP;
      sm.h[e] = (a < rb && q < nf) ? B.h[(size_t)(g0 + a) * nf + q] : 0.f;
    }
    __syncthreads();
    lq = argmax_dequant<H, 32, 32, true>(sm, dq, NoiseSrc{noise, 0, 0}, g0, rb, nf);   // act read per launch
    for (int e = tid; e < rb * nf; e += BLOCK) {
      const int a = e / nf, q = e - a * nf;
      B.h[(size_t)g0 * nf + e] = sm.h[a * NFP + q];
    }
  } else if (kind == ENFLOW_DEQUANT_FLOOR) {
    for (int e = tid; e < rb * nf; e += BLOCK) B.h[(size_t)g0 * nf + e] += scale * noise[(size_t)g0 * nf + e];
  }
  const float s = block_sum(sm, lq);
  if (tid == 0) B.ldj_blk[b] = s;
}

// dequantize.reverse per atom (argmax.py:27-28 / floor.py:13)
__global__ void __launch_bounds__(BLOCK) lg_dequant_rev_kernel(LgArgs B, int kind, int32_t* argmax_idx,
                                                               int32_t* max_idx) {
  const int a = blockIdx.x * BLOCK + threadIdx.x;
  if (a >= B.num_atoms) return;
  const int nf = B.nf;
  float* h = B.h + (size_t)a * nf;
  if (kind == ENFLOW_DEQUANT_ARGMAX) {
    int best = 0;
    float bv = h[0];
    for (int q = 1; q < nf; ++q)
      if (h[q] > bv) { bv = h[q]; best = q; }
    argmax_idx[a] = best;
    atomicMax(max_idx, best);
  } else if (kind == ENFLOW_DEQUANT_FLOOR) {
    for (int q = 0; q < nf; ++q) h[q] = floorf(h[q]);
  }
}

// log|detJ| per molecule (its blocks in order), then the batch total in double
__global__ void __launch_bounds__(BLOCK) lg_ldj_kernel(LgArgs B, float* ldj_mol, double cst, float* total) {
  __shared__ double red[BLOCK];
  const int tid = threadIdx.x;
  double s = 0.0;
  for (int m = tid; m < B.num_mols; m += BLOCK) {
    float v = 0.f;
    for (int b = B.blk_start[m]; b < B.blk_start[m + 1]; ++b) v += B.ldj_blk[b];
    ldj_mol[m] = v;
    s += (double)v;
  }
  red[tid] = s;
  __syncthreads();
  for (int off = BLOCK / 2; off > 0; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  if (tid == 0) total[0] = (float)(red[0] + cst);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static inline hipStream_t LS(void* s) { return reinterpret_cast<hipStream_t>(s); }
static const double kLog2PiL = 1.8378770664093453;

LgWorkspace lg_workspace(int num_mols, int num_atoms, int max_n, int nf) {
  LgWorkspace W;
  const size_t A = (size_t)num_atoms, NB = (size_t)num_atoms / 4 + num_mols + 1;   // blocks of >= 4 rows
  size_t o = 0;
  W.mask = o; o = al256(o + A * 4);
  W.idmap = o; o = al256(o + A * 4);
  W.npairs = o; o = al256(o + A * 4);
  W.cntrow = o; o = al256(o + A * 4);
  W.blk_start = o; o = al256(o + ((size_t)num_mols + 1) * 4);
  W.aabb = o; o = al256(o + (size_t)num_mols * 6 * 4);
  W.ldj_blk = o; o = al256(o + NB * 4);
  W.pos2 = o; o = al256(o + A * 3 * 4);
  W.h2 = o; o = al256(o + A * nf * 4);
  W.pairs = o; o = al256(o + A * (size_t)max_n * 4);
  W.total = o;
  return W;
}

static int lg_check(int num_mols, int num_atoms, int max_n, int nf, int H, int prec) {
  if (num_mols < 0 || num_atoms < 0 || max_n < 0) return -1;
  if (max_n >= (1 << 22)) return -3;   // 22-bit column labels in the pair words
  if (nf < 1 || nf > NFMAX) return -4;
  if (!(H == 32 || H == 64 || H == 128)) return -5;
  const int p = prec & 0xff;
  if ((prec & ~(0xff | ENFLOW_EGCL_VARIANTS)) || p < ENFLOW_PREC_F32 || p > ENFLOW_PREC_BF16) return -1;
  return 0;
}

template <int HH, int PREC>
static void lg_layer_launch(bool var, int grid, hipStream_t st, const LgArgs& B, int mode) {
  if (var) ENFLOW_TIMED("lg_layer_kernel", st, hipLaunchKernelGGL((lg_layer_kernel<HH, PREC, true>), dim3(grid), dim3(BLOCK), 0, st, B, mode));
  else ENFLOW_TIMED("lg_layer_kernel", st, hipLaunchKernelGGL((lg_layer_kernel<HH, PREC, false>), dim3(grid), dim3(BLOCK), 0, st, B, mode));
}
template <int HH>
static void lg_layer_prec(int prec, int grid, hipStream_t st, const LgArgs& B, int mode) {
  const bool var = (prec & ENFLOW_EGCL_VARIANTS) != 0;
  switch (prec & 0xff) {
    case ENFLOW_PREC_F16X3: lg_layer_launch<HH, PREC_F16X3>(var, grid, st, B, mode); break;
    case ENFLOW_PREC_BF16: lg_layer_launch<HH, PREC_BF16>(var, grid, st, B, mode); break;
    default: lg_layer_launch<HH, PREC_F32>(var, grid, st, B, mode); break;
  }
}
static void lg_layer(int H, int prec, int grid, hipStream_t st, const LgArgs& B, int mode) {
  if (H == 32) lg_layer_prec<32>(prec, grid, st, B, mode);
  else if (H == 64) lg_layer_prec<64>(prec, grid, st, B, mode);
  else lg_layer_prec<128>(prec, grid, st, B, mode);
}

// images -> id_mapping -> pair words (reverse: after the pre-network half step)
static void lg_search_rev(hipStream_t st, const LgArgs& B, int rev) {
  const int A = B.num_atoms;
  ENFLOW_TIMED("lg_images_kernel", st, hipLaunchKernelGGL(lg_images_kernel, dim3((A + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, B, rev));
  ENFLOW_TIMED("lg_idmap_kernel", st, hipLaunchKernelGGL(lg_idmap_kernel, dim3(B.num_mols), dim3(IDB), 0, st, B));
  ENFLOW_TIMED("lg_pairs_kernel", st, hipLaunchKernelGGL(lg_pairs_kernel, dim3(lg_grid(B)), dim3(BLOCK), 0, st, B));
}
void lg_search(hipStream_t st, const LgArgs& B) {
  if (B.num_atoms > 0) lg_search_rev(st, B, 0);
}
void lg_setup(hipStream_t st, const LgArgs& B) {
  hipLaunchKernelGGL(lg_setup_kernel, dim3(1), dim3(BLOCK), 0, st, B.mol_ptr, B.num_mols, B.rbl,
                     const_cast<int32_t*>(B.blk_start));
}

// images -> id_mapping -> pair words -> layer, for one layer
static void lg_one_layer(int H, int prec, hipStream_t st, LgArgs& B, int rev, int mode) {
  lg_search_rev(st, B, rev);
  lg_layer(H, prec, lg_grid(B), st, B, mode);
}

// rows per block: the largest of 32 / 16 / 8 / 4 that still gives >= 2
// workgroups per CU (a single 2944-atom box: 4 rows, ~740 blocks; a batch of
// many mid-size molecules: 32).  ENFLOW_LARGE_ROWS overrides (A/B runs).
int lg_rows(int num_atoms) {
  if (const char* e = getenv("ENFLOW_LARGE_ROWS")) {
    const int v = atoi(e);
    if (v == 4 || v == 8 || v == 16 || v == 32) return v;
  }
  for (int r = 32; r > 4; r >>= 1)
    if (num_atoms / r >= 512) return r;
  return 4;
}

LgArgs lg_args(int num_mols, int num_atoms, int max_n, int nf, const int32_t* mol_ptr, const float* r_cut,
                      const float* box, float* h, float* g, float* pos, float* vel, float dt, float cw,
                      int32_t* err, void* ws) {
  const LgWorkspace W = lg_workspace(num_mols, num_atoms, max_n, nf);
  char* base = static_cast<char*>(ws);
  LgArgs B{};
  B.mol_ptr = mol_ptr; B.r_cut = r_cut; B.box = box;
  B.h = h; B.g = g; B.pos = pos; B.vel = vel;
  B.h2 = reinterpret_cast<float*>(base + W.h2);
  B.pos2 = reinterpret_cast<float*>(base + W.pos2);
  B.nf = nf; B.dt = dt; B.cw = cw;
  B.mask = reinterpret_cast<uint32_t*>(base + W.mask);
  B.idmap = reinterpret_cast<int32_t*>(base + W.idmap);
  B.npairs = reinterpret_cast<int32_t*>(base + W.npairs);
  B.cntrow = reinterpret_cast<int32_t*>(base + W.cntrow);
  B.pairs = reinterpret_cast<uint32_t*>(base + W.pairs);
  B.max_n = max_n;
  B.blk_start = reinterpret_cast<int32_t*>(base + W.blk_start);
  B.aabb = reinterpret_cast<float*>(base + W.aabb);
  B.rbl = lg_rows(num_atoms);
  B.ldj_blk = reinterpret_cast<float*>(base + W.ldj_blk);
  B.err = err;
  B.num_mols = num_mols; B.num_atoms = num_atoms;
  return B;
}

extern "C" {

int64_t enflow_lf_large_workspace_size(int num_mols, int num_atoms, int max_mol_atoms, int nf) {
  if (num_mols < 0 || num_atoms < 0 || max_mol_atoms < 0 || nf < 1 || nf > NFMAX) return -1;
  return (int64_t)lg_workspace(num_mols, num_atoms, max_mol_atoms, nf).total;
}

int enflow_lf_forward_large_f32(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                                const int32_t* mol_ptr, const float* r_cut, const float* box,
                                float* h, float* g, float* pos, float* vel,
                                const float* layers, int n_layers,
                                int dequant_kind, const float* dequant, const float* noise,
                                float dequant_scale, float dt, float cw,
                                float* ldj_mol, float* ldj_total, int32_t* err_flag, int gemm_precision,
                                float* tape, int32_t* pair_rows,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = lg_check(num_mols, num_atoms, max_mol_atoms, nf, H, gemm_precision);
  if (rc) return rc;
  if (n_layers < 0 || (dequant_kind != ENFLOW_DEQUANT_NONE && !noise) ||
      (dequant_kind == ENFLOW_DEQUANT_ARGMAX && !dequant) || !workspace || !ldj_mol || !ldj_total || !err_flag)
    return -1;
  // the tape feeds the fp32-accurate backward (enflow_lf_backward_large_f32)
  if (tape && (!pair_rows || (gemm_precision & 0xff) == ENFLOW_PREC_BF16)) return -1;
  if (workspace_bytes < enflow_lf_large_workspace_size(num_mols, num_atoms, max_mol_atoms, nf)) return -6;
  const hipStream_t st = LS(stream);
  LgArgs B = lg_args(num_mols, num_atoms, max_mol_atoms, nf, mol_ptr, r_cut, box, h, g, pos, vel, dt, cw,
                     err_flag, workspace);
  const int grid_blk = lg_grid(B);
  B.tape = tape;
  B.pair_rows = pair_rows;
  B.n_layers = n_layers;
  if (tape && n_layers > 0 && hipMemsetAsync(pair_rows, 0, (size_t)n_layers * 4, st) != hipSuccess) return -2;
  if (num_mols > 0) {
    lg_setup(st, B);
    if (H == 32) hipLaunchKernelGGL((lg_dequant_kernel<32>), dim3(grid_blk), dim3(BLOCK), 0, st, B, dequant_kind, dequant, noise, dequant_scale);
    else if (H == 64) hipLaunchKernelGGL((lg_dequant_kernel<64>), dim3(grid_blk), dim3(BLOCK), 0, st, B, dequant_kind, dequant, noise, dequant_scale);
    else hipLaunchKernelGGL((lg_dequant_kernel<128>), dim3(grid_blk), dim3(BLOCK), 0, st, B, dequant_kind, dequant, noise, dequant_scale);
    const size_t stride = egcl_layout(H, nf).total;
    float *cur_h = h, *cur_pos = pos, *nxt_h = B.h2, *nxt_pos = B.pos2;
    for (int l = 0; l < n_layers; ++l) {
      B.layer = layers + (size_t)l * stride;
      B.layer_idx = l;
      B.h = cur_h; B.pos = cur_pos; B.h2 = nxt_h; B.pos2 = nxt_pos;
      lg_one_layer(H, gemm_precision, st, B, 0, 0);
      float* t = cur_h; cur_h = nxt_h; nxt_h = t;
      t = cur_pos; cur_pos = nxt_pos; nxt_pos = t;
    }
    if (cur_h != h) {
      if (hipMemcpyAsync(h, cur_h, (size_t)num_atoms * nf * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) return -2;
      if (hipMemcpyAsync(pos, cur_pos, (size_t)num_atoms * 3 * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) return -2;
    }
  }
  const double cst = dequant_kind == ENFLOW_DEQUANT_ARGMAX ? -0.5 * kLog2PiL : 0.0;
  hipLaunchKernelGGL(lg_ldj_kernel, dim3(1), dim3(BLOCK), 0, st, B, ldj_mol, cst, ldj_total);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int enflow_lf_reverse_large_f32(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                                const int32_t* mol_ptr, const float* r_cut, const float* box,
                                float* h, float* g, float* pos, float* vel,
                                const float* layers, int n_layers,
                                int dequant_kind, float dt, float cw,
                                int32_t* argmax_idx, int32_t* max_idx, int32_t* err_flag, int gemm_precision,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = lg_check(num_mols, num_atoms, max_mol_atoms, nf, H, gemm_precision);
  if (rc) return rc;
  if (n_layers < 0 || (dequant_kind == ENFLOW_DEQUANT_ARGMAX && (!argmax_idx || !max_idx)) || !workspace ||
      !err_flag)
    return -1;
  if (workspace_bytes < enflow_lf_large_workspace_size(num_mols, num_atoms, max_mol_atoms, nf)) return -6;
  const hipStream_t st = LS(stream);
  LgArgs B = lg_args(num_mols, num_atoms, max_mol_atoms, nf, mol_ptr, r_cut, box, h, g, pos, vel, dt, cw,
                     err_flag, workspace);
  if (num_mols > 0) {
    hipLaunchKernelGGL(lg_setup_kernel, dim3(1), dim3(BLOCK), 0, st, mol_ptr, num_mols, B.rbl, B.blk_start);
    const size_t stride = egcl_layout(H, nf).total;
    for (int it = 0; it < n_layers; ++it) {
      B.layer = layers + (size_t)(n_layers - 1 - it) * stride;
      lg_one_layer(H, gemm_precision, st, B, 1, 1);
    }
    if (num_atoms > 0)
      hipLaunchKernelGGL(lg_dequant_rev_kernel, dim3((num_atoms + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, B,
                         dequant_kind, argmax_idx, max_idx);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int enflow_egcl_forward_large_f32(int num_mols, int num_atoms, int max_mol_atoms, int nf, int H,
                                  const int32_t* mol_ptr, const float* r_cut, const float* box,
                                  const float* h, const float* pos, const float* layer, float cw,
                                  float* Q, float* F, float* G, int32_t* err_flag, int gemm_precision,
                                  void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = lg_check(num_mols, num_atoms, max_mol_atoms, nf, H, gemm_precision);
  if (rc) return rc;
  if (!workspace || !err_flag || !layer || !Q || !F || !G) return -1;
  if (workspace_bytes < enflow_lf_large_workspace_size(num_mols, num_atoms, max_mol_atoms, nf)) return -6;
  const hipStream_t st = LS(stream);
  LgArgs B = lg_args(num_mols, num_atoms, max_mol_atoms, nf, mol_ptr, r_cut, box, const_cast<float*>(h), nullptr,
                     const_cast<float*>(pos), nullptr, 0.f, cw, err_flag, workspace);
  B.layer = layer;
  B.Qo = Q; B.Fo = F; B.Go = G;
  if (num_mols > 0) {
    hipLaunchKernelGGL(lg_setup_kernel, dim3(1), dim3(BLOCK), 0, st, mol_ptr, num_mols, B.rbl, B.blk_start);
    lg_one_layer(H, gemm_precision, st, B, 0, 2);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int enflow_neighbour_pairs_large_f32(int num_mols, int num_atoms, int max_mol_atoms, const int32_t* mol_ptr,
                                     const float* r_cut, const float* box, const float* pos, int32_t* npairs,
                                     uint32_t* pairs, int32_t* err_flag, void* workspace, int64_t workspace_bytes,
                                     void* stream) {
  int rc = lg_check(num_mols, num_atoms, max_mol_atoms, 1, 32, ENFLOW_PREC_F32);
  if (rc) return rc;
  if (!workspace || !err_flag || !npairs || !pairs) return -1;
  if (workspace_bytes < enflow_lf_large_workspace_size(num_mols, num_atoms, max_mol_atoms, 1)) return -6;
  const hipStream_t st = LS(stream);
  LgArgs B = lg_args(num_mols, num_atoms, max_mol_atoms, 1, mol_ptr, r_cut, box, nullptr, nullptr,
                     const_cast<float*>(pos), nullptr, 0.f, 0.f, err_flag, workspace);
  B.npairs = npairs;
  B.pairs = pairs;
  if (num_mols > 0 && num_atoms > 0) {
    hipLaunchKernelGGL(lg_images_kernel, dim3((num_atoms + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, B, 0);
    hipLaunchKernelGGL(lg_idmap_kernel, dim3(num_mols), dim3(IDB), 0, st, B);
    hipLaunchKernelGGL(lg_setup_kernel, dim3(1), dim3(BLOCK), 0, st, mol_ptr, num_mols, B.rbl, B.blk_start);
    hipLaunchKernelGGL(lg_pairs_kernel, dim3(num_atoms / B.rbl + num_mols + 1), dim3(BLOCK), 0, st, B);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
