// flow_kernel.h -- the fused flow kernel (forward or reverse), shared by the
// 256-thread build (enflow_flow.hip: one workgroup of 4 waves per molecule, two
// workgroups per CU) and the latency build (enflow_latency.hip: 8 waves per
// molecule, one workgroup per CU, for batches that do not fill the chip).
// Included after flow_device.h; WAVES / BLOCK come from the including TU.
#pragma once

// ---------------------------------------------------------------------------
// the fused flow kernel (forward or reverse)
// ---------------------------------------------------------------------------
#ifndef ENFLOW_BLOCKED_WPS
#define ENFLOW_BLOCKED_WPS ENFLOW_WAVES_PER_SIMD   // row-blocked (> 64-atom) instances
#endif
// batch log|detJ| in the same launch: every workgroup publishes its ldj_mol
// entry and takes a ticket; the last one sums ldj_mol in reduce_ldj_kernel's
// fixed order (per-thread strided double sums, then a tree over the block) --
// bitwise the separate reduction's result -- and resets the ticket for the
// next launch on the stream.  `red` is 256 doubles of LDS scratch.
__device__ __forceinline__ void ticket_reduce_ldj(const FlowArgs& A, double* red, int* last) {
  const int tid = threadIdx.x;
  __threadfence();                       // this block's ldj_mol entry visible device-wide
  __syncthreads();
  if (tid == 0) *last = atomicAdd(A.ticket, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!*last) return;
  __threadfence();                       // acquire: every block's entry
  // the first RT = 256 threads, whatever the block size: the same order as
  // reduce_ldj_kernel in every instance
  constexpr int RT = 256;
  double s = 0.0;
  if (tid < RT)
    for (int m = tid; m < A.num_mols; m += RT) s += (double)__builtin_nontemporal_load(&A.ldj_mol[m]);
  if (tid < RT) red[tid] = s;
  __syncthreads();
  for (int off = RT / 2; off > 0; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  if (tid == 0) {
    A.ldj_total[0] = (float)(red[0] + A.ldj_cst);
    atomicExch(A.ticket, 0u);
  }
}

// FDQ = false: an instance without the fused ArgMax dequantisation, for launches
// whose dequantisation ran ahead (dequant_kernel) or is Floor / none -- the
// unused ArgMax path otherwise costs the layer loop ~1.4 % in code generation
// (profiles/r06/r06n_*: 0.7099 ms with it, ~0.700 without)
template <int H, int NMAX, bool REV, int PREC, int RB, bool VAR, bool FDQ = true>
__global__ void __launch_bounds__(BLOCK, (RB < NMAX ? ENFLOW_BLOCKED_WPS : ENFLOW_WAVES_PER_SIMD))
    lf_flow_kernel(FlowArgs A) {
  __shared__ Smem<H, NMAX, RB> sm;
  constexpr bool BLOCKED = RB < NMAX;
  MolRef M;
#ifdef ENFLOW_PRIO
  // A/B: static issue priority for one of the two workgroups sharing a CU
  if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(ENFLOW_PRIO);
#endif
  STAMP_DECL
#ifdef ENFLOW_SKEW
  // A/B experiment: offset the second resident workgroup of a CU so the two
  // molecules' serial phases (pair build, node phase) overlap the other's tiles
  if (blockIdx.x & ENFLOW_SKEW_BIT)
    {
#pragma unroll
      for (int i = 0; i < ENFLOW_SKEW; ++i) __builtin_amdgcn_s_sleep(127);
    }
#endif
  if (!load_molecule(sm, A, M, LOAD_POS | LOAD_H | LOAD_VELG)) {   // error raised; keep the ticket count
    if (!REV && A.ticket) {
      if (threadIdx.x == 0) A.ldj_mol[M.m] = 0.f;
      ticket_reduce_ldj(A, reinterpret_cast<double*>(sm.agg), &sm.npairs);
    }
    return;
  }
  STAMP(0);
  const int tid = threadIdx.x;
  const int n = M.n, nf = A.nf;
  const EgclLayout L = egcl_layout(H, nf);
  constexpr int AST = Smem<H, NMAX, RB>::AST;
  float ldj = 0.f;
  // per-atom pbc box (Data.pbc, base.py): LDS image, or global memory when blocked
  auto pbox = [&](int a, int d) {
    if constexpr (BLOCKED) return A.box[((size_t)M.a0 + a) * 3 + d];
    else return sm.boxa[a * 3 + d];
  };

  if (!REV) {
    if (FDQ && A.dequant_kind == ENFLOW_DEQUANT_ARGMAX) {
      if constexpr (FDQ) ldj += argmax_dequant<H, NMAX, RB, VAR>(sm, A.dequant, A.noise_src(), M.a0, n, nf);
    } else if (A.dequant_kind == ENFLOW_DEQUANT_FLOOR) {
      for (int e = tid; e < n * nf; e += BLOCK) {
        const int a = e / nf, q = e - a * nf;
        sm.h[a * NFP + q] += A.dequant_scale * A.noise_src().uniform((size_t)M.a0 * nf + e);
      }
      __syncthreads();
    }
  }
  STAMP(1);

  for (int it = 0; it < A.n_layers; ++it) {
    // Opaque per-layer copies: stop hipcc from hoisting every nf / molecule
    // derived predicate and address out of the layer loop (SGPR/VGPR spills).
    int nf = __builtin_amdgcn_readfirstlane(A.nf), n = __builtin_amdgcn_readfirstlane(M.n), tid_l = tid;
    asm volatile("" : "+s"(nf), "+s"(n), "+v"(tid_l));
    MolRef Ml = M;
    Ml.n = n;
    const EgclLayout L = egcl_layout(H, nf);
    const int l = REV ? A.n_layers - 1 - it : it;
    const float* Lp = A.layers + (size_t)l * L.total;
    if (REV) {   // dynamics.py:28-30
      for (int a = tid; a < n; a += BLOCK) {
        for (int q = 0; q < nf; ++q) sm.h[a * NFP + q] -= sm.g[a * NFP + q] * A.dt;
        for (int d = 0; d < 3; ++d)
          sm.pos[a * 3 + d] = pbc1(sm.pos[a * 3 + d] - sm.vel[a * 3 + d] * A.dt, pbox(a, d));
      }
      __syncthreads();
    }
    build_images(sm, Ml, tid_l);
    STAMP(3);
    int npairs_layer = 0;
    auto block_pass = [&](const int r0, const int rb) {
      int tot;
      if constexpr (BLOCKED) {
        block_counts(sm, Ml, tid_l, r0, rb);
        tot = block_compact(sm, n, tid_l, rb, 0);
      } else {
        build_block_pairs(sm, Ml, tid_l, r0, rb);
        tot = sm.npairs;
      }
      STAMP(2);
      npairs_layer += tot;
      if (A.stats != nullptr && tid == 0) {
        unsigned long long edges = 0;
        for (int a = 0; a < rb; ++a) edges += (unsigned long long)sm.cntrow[r0 + a];
        atomicAdd(&A.stats[0], (unsigned long long)tot);
        atomicAdd(&A.stats[1], edges);
      }
      // the node phase's first fragments, requested as each wave leaves its tiles
      // (the whole-molecule split-precision image: one edge_tiles pass per layer)
      NodeFrags<H> nfr;
      constexpr bool EARLY = !BLOCKED && PREC != PREC_F32;
      const int wv = __builtin_amdgcn_readfirstlane(tid_l >> 6);
      auto pre = [&] {
        if constexpr (EARLY) {
          if (wv < (H / 32) * (RB / 32)) nfr.issue(weights_rsrc(Lp, L.total), L, tid_l & 63, wv);
        }
      };
      edge_tiles<H, NMAX, RB, PREC, VAR>(sm, Lp, L, Ml, nf, tid_l, r0, rb, true STAMP_PASS, nullptr, nullptr, pre);
      if constexpr (BLOCKED) {   // blocks with more pairs than the buffer: further passes
        constexpr int PC = Smem<H, NMAX, RB>::PC;
        for (int p0 = PC; p0 < tot; p0 += PC) {
          block_compact(sm, n, tid_l, rb, p0);
          edge_tiles<H, NMAX, RB, PREC, VAR>(sm, Lp, L, Ml, nf, tid_l, r0, rb, false STAMP_PASS);
        }
      }
      STAMP(4);
      {
        if constexpr (PREC != PREC_F32)   // fp32-accurate
          node_phase_x3_f<H, NMAX, RB, VAR>(sm, Lp, L, n, nf, tid_l, r0, rb, nfr, EARLY);
        else node_phase<H, NMAX, RB, VAR>(sm, Lp, L, n, nf, tid_l, r0, rb);
      }
      STAMP(5);
      if constexpr (PREC == PREC_F16X3) {   // every F16X3 operand kind saw a value >= 2^-7 (BIGK_*)?
        if (tid == 0) {
          if (small_operands(sm.big)) sm.err |= ENFLOW_ERR_SMALL;
          sm.big = 0u;   // next written after this layer's / block's barriers
        }
      }
      if (!REV && A.tape != nullptr) {   // training tape: layer-input state + message sums + Q
        const TapeLayout T = tape_layout(A.num_atoms, nf, H, A.n_layers);
        const size_t la = (size_t)l * A.num_atoms + M.a0 + r0;
        float* hx = A.tape + T.hx + la * T.ldhx;
        for (int e = tid; e < rb * T.ldhx; e += BLOCK) {
          const int a = e / T.ldhx, c = e - a * T.ldhx;
          hx[e] = c < nf ? sm.h[(r0 + a) * NFP + c] : sm.agg[a * AST + (c - nf)];
        }
        for (int e = tid; e < rb * nf; e += BLOCK) {
          const int a = e / nf, q = e - a * nf;
          A.tape[T.g + la * nf + e] = sm.g[(r0 + a) * NFP + q];
        }
        for (int e = tid; e < rb * 3; e += BLOCK) {
          A.tape[T.pos + la * 3 + e] = sm.pos[r0 * 3 + e];
          A.tape[T.vel + la * 3 + e] = sm.vel[r0 * 3 + e];
        }
        for (int a = tid; a < rb; a += BLOCK) A.tape[T.q + la + a] = sm.Q[r0 + a];
        // the layer's neighbour list for the backward: the 64-atom image only (the
        // training forward's instance for molecules of 33..64 atoms; the <= 32-atom
        // instances keep their registers -- their backward rebuilds the list)
        if constexpr (!BLOCKED && NMAX == TAPE_PAIR_CAP + 1) {
          float* const tp = A.tape + T.pairs + la * TAPE_PAIR_CAP;
          for (int e = tid; e < sm.npairs; e += BLOCK) tp[e] = __uint_as_float(sm.pairs[e]);
          for (int a = tid; a < rb; a += BLOCK) A.tape[T.cnt + la + a] = __int_as_float(sm.cntrow[r0 + a]);
        }
        __syncthreads();   // every thread's copy done before the leapfrog update rewrites pos / vel / h / g
      }
      if constexpr (BLOCKED) {   // park the block's forces (egcl.py:73-74)
        for (int e = tid; e < rb * 3; e += BLOCK) {
          const int a = e / 3, d = e - a * 3;
          const float inv = 1.f / fmaxf((float)sm.cntrow[r0 + a], 1.f);
          sm.F[(r0 + a) * 3 + d] = sm.agg[a * AST + H + d] * inv * A.cw;
        }
        __syncthreads();
      }
    };
    if constexpr (BLOCKED) {
      for (int r0 = 0; r0 < n; r0 += RB) block_pass(r0, min(RB, n - r0));
    } else {
      block_pass(0, n);   // the whole molecule in one pass
    }
    if (!REV && A.tape != nullptr && tid == 0 && A.pair_counts != nullptr)
      A.pair_counts[(size_t)l * A.num_mols + M.m] = npairs_layer;
    for (int a = tid; a < n; a += BLOCK) {
      const float q = sm.Q[a];
      const float eq = expf(q);
      const float inv = 1.f / fmaxf((float)sm.cntrow[a], 1.f);   // helpers.py:63-70
      auto force = [&](int d) {
        if constexpr (BLOCKED) return sm.F[a * 3 + d];
        else return sm.agg[a * AST + H + d] * inv * A.cw;
      };
      if (!REV) {  // dynamics.py:15-22
        for (int d = 0; d < 3; ++d) {
          const float F = force(d);
          const float v = eq * sm.vel[a * 3 + d] + F * A.dt;
          sm.vel[a * 3 + d] = v;
          sm.pos[a * 3 + d] = pbc1(sm.pos[a * 3 + d] + v * A.dt, pbox(a, d));
        }
        for (int qf = 0; qf < nf; ++qf) {
          const float gn = sm.g[a * NFP + qf] + sm.G[a * NFP + qf] * A.dt;
          sm.g[a * NFP + qf] = gn;
          sm.h[a * NFP + qf] += gn * A.dt;
        }
        ldj += q;
      } else {     // dynamics.py:32-35
        for (int qf = 0; qf < nf; ++qf) sm.g[a * NFP + qf] -= sm.G[a * NFP + qf] * A.dt;
        for (int d = 0; d < 3; ++d) {
          const float F = force(d);
          sm.vel[a * 3 + d] = (sm.vel[a * 3 + d] - F * A.dt) / eq;
        }
      }
    }
    __syncthreads();
    STAMP(6);
  }

  if (REV) {   // dequantize.reverse (argmax.py:27-28 / floor.py:13)
    for (int a = tid; a < n; a += BLOCK) {
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
    __syncthreads();   // the write-back below maps threads to elements differently
  }
  // write back.  Split-precision GEMMs (f16x3 / bf16) cannot represent operands
  // past the fp16 / bf16 range: a non-finite output they produce is flagged
  // (ENFLOW_ERR_RANGE) instead of returned silently; the f32 path returns
  // whatever the arithmetic gives, as the reference does.
  bool bad = false;
  for (int e = tid; e < n * 3; e += BLOCK) {
    const float p = sm.pos[e], v = sm.vel[e];
    A.pos[(size_t)M.a0 * 3 + e] = p;
    A.vel[(size_t)M.a0 * 3 + e] = v;
    bad |= !__builtin_isfinite(p) || !__builtin_isfinite(v);
  }
  for (int e = tid; e < n * nf; e += BLOCK) {
    const int a = e / nf, q = e - a * nf;
    const float hv = sm.h[a * NFP + q], gv = sm.g[a * NFP + q];
    A.h[(size_t)M.a0 * nf + e] = hv;
    A.g[(size_t)M.a0 * nf + e] = gv;
    bad |= (!REV && !__builtin_isfinite(hv)) || !__builtin_isfinite(gv);
  }
  if constexpr (PREC != PREC_F32) {
    if (bad) atomicOr(&sm.err, ENFLOW_ERR_RANGE);
  }
  bad = false;
  if (!REV) {
    float s = block_sum(sm, ldj);   // (its barriers also order the err bits above)
    // dequantised ahead (dequant_kernel): its log_q, read here rather than at
    // the start (the read there cost the layer loop ~3 % in register allocation,
    // profiles/r06/r06l_*)
    if (A.lq_mol != nullptr) s += A.lq_mol[M.m];
    if (tid == 0) A.ldj_mol[M.m] = s;
    bad = tid == 0 && !__builtin_isfinite(s);
  } else {
    __syncthreads();
  }
  if (tid == 0) {
    const int e = sm.err | ((PREC != PREC_F32 && bad) ? ENFLOW_ERR_RANGE : 0);
    if (e) {
      atomicOr(A.err, e);
      if (A.mol_err) atomicOr(&A.mol_err[M.m], e);
    }
  }
  if (!REV && A.ticket) ticket_reduce_ldj(A, reinterpret_cast<double*>(sm.agg), &sm.npairs);
  STAMP(7);
  STAMP_FLUSH
}

