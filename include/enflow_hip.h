/*
 * enflow_hip.h -- C ABI of the MI355X (gfx950) coupling-flow hot path.
 *
 * The reference (bharath-raghavan/enflow) is pure Python/PyTorch; it has no
 * FFI.  Each entry point below replaces one operator of the reference's
 * nn.Module surface (cited per function) and is bound from Python with ctypes
 * by enflow_amd/_lib.py (see INTEGRATION.md for the binding a maintainer of the
 * reference would add).
 *
 * Conventions
 *   - every pointer is a DEVICE pointer (hipMalloc / torch CUDA storage) unless
 *     documented otherwise; sizes are element counts;
 *   - a batch is the concatenation of molecules (the reference's Data layout,
 *     enflow/data/base.py:21-50): mol_ptr[num_mols + 1] (int32) holds the
 *     atom offsets, per-atom arrays are row-major [num_atoms][k];
 *   - stream is a hipStream_t passed as void* (NULL = default stream);
 *   - return value 0 = launched, < 0 = argument error (nothing launched);
 *     data-dependent faults the reference would raise on (e.g. fewer periodic
 *     images than atoms) are reported through err_flag (device int32, OR-ed
 *     ENFLOW_ERR_* bits) which the host reads after the stream syncs.
 *   - max_mol_atoms is the largest molecule in the batch (host-known from
 *     Data.N); it selects the kernel instantiation (<= 32, <= 64 or <= 256
 *     atoms; larger systems go through the *_large_* entry points);
 *   - all arithmetic is float32 (the reference computes in float64; parity is
 *     1e-5 relative).
 */
#ifndef ENFLOW_HIP_H
#define ENFLOW_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ENFLOW_ERR_TOO_MANY_ATOMS   1  /* molecule larger than the kernel's NMAX */
#define ENFLOW_ERR_FEW_IMAGES       2  /* reference would IndexError (base.py:137) */
#define ENFLOW_ERR_TOO_MANY_FEATURES 4
#define ENFLOW_ERR_RANGE            8  /* f16x3 / bf16 GEMM path produced a non-finite output
                                          (an operand past the fp16 / bf16 range): rerun with
                                          ENFLOW_PREC_F32 */
#define ENFLOW_ERR_SMALL           16  /* ABI 12 (ABI 11 reported it as ENFLOW_ERR_RANGE): an f16x3 GEMM
                                          operand of a molecule / row block was entirely below 2^-7
                                          in magnitude (its fp16 lo parts subnormal, ~1e-5 relative
                                          error): a precision warning, not an overflow; rerun with
                                          ENFLOW_PREC_F32 for the fp32-accurate result */
#define ENFLOW_ERR_HANDOFF         32  /* ABI 12: a two-workgroup latency launch (enflow_set_split_threshold)
                                          timed out waiting for its partner workgroup (not co-resident):
                                          outputs invalid, rerun with the split instance off */

/* Precision of the flow's two H x H edge GEMMs (edge_nn.2, coord_nn.0); all
 * other arithmetic is fp32 in every mode.  See DESIGN.md for the error model. */
#define ENFLOW_PREC_F32   0  /* v_mfma_f32_32x32x2_f32: exact fp32 FMA chain          */
#define ENFLOW_PREC_F16X3 1  /* fp32 operands split hi+lo in fp16, 3 products, fp32 acc */
#define ENFLOW_PREC_BF16  2  /* bf16 operands, fp32 accumulation                       */
/* ABI 13: OR into gemm_precision of the forward / reverse io / io2 entries: the
 * launch does not take the feature-split instances (enflow_set_split_threshold /
 * enflow_set_fs_threshold) whatever the thresholds say -- the per-call re-run
 * after ENFLOW_ERR_HANDOFF, without touching the process-wide setting. */
#define ENFLOW_PREC_NO_SPLIT 0x400

#define ENFLOW_DEQUANT_NONE   0
#define ENFLOW_DEQUANT_ARGMAX 1  /* enflow/nn/argmax.py */
#define ENFLOW_DEQUANT_FLOOR  2  /* enflow/nn/floor.py  */

/* ABI version of this header; bump on any signature or error-semantics change (6: ENFLOW_ERR_RANGE,
 * bf16 + tape rejected, NaN-poisoned gradients on a backward error, enflow_timing_*; 7: training
 * on large systems -- tape / pair_rows of enflow_lf_forward_large_f32, enflow_lf_backward_large_f32,
 * enflow_alchemical_nll_backward_f32 for any molecule size; 8: out-of-place, self-contained
 * forward / reverse -- enflow_lf_forward_io_f32 (in-kernel dequantiser draws, in-launch
 * log|detJ| reduction), enflow_lf_reverse_io_f32; 9: ENFLOW_ERR_RANGE also flagged for a
 * non-finite phi / attention logit before tanh / clamp / sigmoid, the clamp passes NaN like
 * torch.clamp, latency instances of the fused flow kernel, enflow_set_latency_threshold; 10: act_fn
 * kinds (enflow_pack_egcl_act_f32, the ArgMax activation trailer), node_nf up to 16 in
 * libenflow_hip_nf16.so; 11: ENFLOW_ERR_RANGE also flags an f16x3 GEMM operand that is entirely
 * small, ENFLOW_BWD_F32 -- the fp32-GEMM backward for a tape recorded by an ENFLOW_PREC_F32
 * forward); 12: ENFLOW_ERR_SMALL split from ENFLOW_ERR_RANGE, ENFLOW_ERR_HANDOFF, the feature-split
 * latency instance (enflow_set_split_threshold / enflow_set_fs_threshold), per-molecule error words
 * and molecule lists (enflow_lf_forward_io2_f32 / enflow_lf_reverse_io2_f32); 13: ENFLOW_PREC_NO_SPLIT,
 * enflow_set_handoff_spin_limit, the two-workgroup split only for out-of-place launches, the ArgMax
 * dequantisation ahead of the flow kernel, enflow_set_dequant_ahead, enflow_pack_egcl_layers_f32 /
 * enflow_pack_egcl_bwd_layers_f32). */
int enflow_abi_version(void);

/* Batches of <= 32-atom molecules with at most this many molecules run the
 * fused flow kernel's latency instance (8 waves per molecule, one workgroup
 * per CU) instead of the 4-wave one (two per CU).  -1 (default): the current
 * device's CU count.  Replaces no reference interface: the reference has no
 * kernels; this is the strong-scaling knob of enflow/main.py:141-145's
 * DistributedSampler split (a fixed batch over more GPUs = fewer molecules per
 * GPU).  Returns the previous setting; enflow_latency_threshold() returns the
 * one in effect on the current device. */
int enflow_set_latency_threshold(int max_mols);
int enflow_latency_threshold(void);

/* ABI 12: the feature-split latency instance (H = 128, f16x3, inference): the
 * eight waves of a workgroup share every 32-pair edge tile in a two-stage
 * pipeline (four per stage), each owning 32 output features of its stage's
 * GEMMs with those weights in registers.  Batches of at most
 * `max_mols` molecules that fit two workgroups per molecule on the device's
 * CUs run it with each molecule's rows split over two workgroups (one position
 * / feature hand-off per layer; -1 (default): CUs / 2; 0: never).
 * enflow_set_fs_threshold: batches of at most `max_mols` molecules that do not
 * take that split run it with one workgroup per molecule (-1 (default): the
 * device's CU count, one round of workgroups; 0: never).
 * Same strong-scaling role as enflow_set_latency_threshold (enflow/main.py:
 * 141-145); both return the previous setting.
 * ABI 13: the two-workgroup split runs only out of place (h_in, g_in, pos_in,
 * vel_in all non-NULL): in place, the two halves of a molecule would read rows
 * the partner may already have overwritten (one-layer flows have no hand-off
 * to order them), so such launches take one workgroup per molecule. */
int enflow_set_split_threshold(int max_mols);
int enflow_set_fs_threshold(int max_mols);
/* ABI 13: polls a waiting workgroup of the two-workgroup split makes for one
 * partner granule before it gives up (ENFLOW_ERR_HANDOFF; once one wait of a
 * workgroup has given up, its later waits give up at once).  Default (-1):
 * 2^20, ~0.1 s.  0: every wait gives up without polling -- forces the
 * ENFLOW_ERR_HANDOFF path, for testing the host's re-run.  Per library;
 * returns the previous setting. */
int enflow_set_handoff_spin_limit(int polls);
/* ABI 13: the ArgMax dequantisation (argmax.py:13-25) of forward io / io2
 * launches on batches of <= 64-atom molecules runs as its own kernel ahead of
 * the flow kernel (one workgroup per molecule, all molecules in parallel; the
 * same draws and values as the fused form, log|detJ| within round-off of
 * it).  1 (default) on, 0 the dequantisation fused into the flow kernel.  Per
 * library; returns the previous setting. */
int enflow_set_dequant_ahead(int on);

/* Largest molecule (atoms) / node_nf the compiled kernels accept.  The ABI
 * ships as two builds of the same sources: libenflow_hip.so (node_nf <= 8) and
 * libenflow_hip_nf16.so (-DENFLOW_NFMAX=16: node_nf <= 16 for inference and
 * for the training / EGCL backward entry points -- since ABI 11 the radial row
 * of the backward's transposed edge_nn.0 GEMM, past its 32-row tile at node_nf
 * 16, is a separate dot); the host picks by node_nf.  The
 * reference sizes EGCL / ArgMax by the dataset's node_nf
 * (enflow/main.py:148-151). */
int enflow_max_atoms(void);
int enflow_max_node_nf(void);
/* 1 if hidden_nf is one of the compiled widths (32, 64, 128). */
int enflow_supports_hidden(int hidden_nf);

/* Floats needed to hold one packed EGCL layer / one packed ArgMax network. */
int64_t enflow_egcl_packed_size(int hidden_nf, int node_nf);
int64_t enflow_argmax_packed_size(int hidden_nf, int node_nf);

/*
 * Pack one EGCL layer's parameters (torch nn.Linear layouts, concatenated in
 * named_parameters() order of enflow/nn/egcl.py:12-55 with the default flags:
 *   edge_nn.0.weight [H][2nf+1], edge_nn.0.bias [H], edge_nn.2.weight [H][H],
 *   edge_nn.2.bias [H], node_nn.0.weight [H][H+nf], node_nn.0.bias [H],
 *   node_nn.2.weight [nf][H], node_nn.2.bias [nf], coord_nn.0.weight [H][H],
 *   coord_nn.0.bias [H], coord_nn.2.weight [1][H], vel_scaling_nn.0.weight
 *   [H][nf], vel_scaling_nn.0.bias [H], vel_scaling_nn.2.weight [1][H],
 *   vel_scaling_nn.2.bias [1])
 * into the MFMA-fragment layout the flow kernels read.
 */
int enflow_pack_egcl_f32(const float* raw, int hidden_nf, int node_nf,
                         float* packed, void* stream);

/* EGCL constructor variants (enflow/nn/egcl.py:11-17, 40-49, 57-63, 80-84). */
#define ENFLOW_EGCL_ATTENTION 1   /* edge messages *= sigmoid(att_nn(messages)) */
#define ENFLOW_EGCL_NORM_DIFF 2   /* force uses coord_diff / (|coord_diff| + 1) */
#define ENFLOW_EGCL_TANH      4   /* phi = tanh(coord_nn(...)) */
#define ENFLOW_EGCL_ACT       8   /* act_fn is not SiLU (egcl.py:11): kind + parameters packed */
/* OR into gemm_precision of enflow_lf_forward_f32 / enflow_lf_reverse_f32 when
 * any layer carries ENFLOW_EGCL_* flags (selects the variant-capable kernels;
 * without it the flags in the packed layers are ignored). */
#define ENFLOW_EGCL_VARIANTS 0x100

/* enflow_pack_egcl_f32 for a layer built with attention / norm_diff / tanh:
 * `raw` in the same (default-flag) order as above, `flags` ENFLOW_EGCL_*,
 * `att` = att_nn.0.weight [1][H] followed by att_nn.0.bias [1] (required with
 * ENFLOW_EGCL_ATTENTION, else ignored).  The flow / EGCL forward and reverse
 * kernels read the flags from the packed layer, the training backward too
 * (see enflow_lf_backward_f32). */
int enflow_pack_egcl_ex_f32(const float* raw, int hidden_nf, int node_nf, int flags,
                            const float* att, float* packed, void* stream);

/* Activations (act_fn of EGCL / ArgMax, enflow/nn/egcl.py:11, argmax.py:7):
 * the torch module's elementwise function, with up to two parameters (p0, p1)
 * as listed.  Forward and derivative definitions: flow_device.h (act_f / act_d). */
#define ENFLOW_ACT_SILU        0
#define ENFLOW_ACT_RELU        1
#define ENFLOW_ACT_LEAKY_RELU  2   /* p0 = negative_slope */
#define ENFLOW_ACT_ELU         3   /* p0 = alpha */
#define ENFLOW_ACT_CELU        4   /* p0 = alpha */
#define ENFLOW_ACT_SELU        5
#define ENFLOW_ACT_GELU        6   /* approximate='none' (erf) */
#define ENFLOW_ACT_GELU_TANH   7   /* approximate='tanh' */
#define ENFLOW_ACT_TANH        8
#define ENFLOW_ACT_SIGMOID     9
#define ENFLOW_ACT_SOFTPLUS   10   /* p0 = beta, p1 = threshold */
#define ENFLOW_ACT_MISH       11
#define ENFLOW_ACT_HARDTANH   12   /* p0 = min_val, p1 = max_val (ReLU6 = 0, 6) */
#define ENFLOW_ACT_IDENTITY   13

/* enflow_pack_egcl_ex_f32 with the layer's act_fn (ABI 10): `flags` carries
 * ENFLOW_EGCL_ACT exactly when act_kind != ENFLOW_ACT_SILU; every launch on
 * such layers ORs ENFLOW_EGCL_VARIANTS into its precision / dequant word (the
 * variant-capable kernels read the activation from the packed layer). */
int enflow_pack_egcl_act_f32(const float* raw, int hidden_nf, int node_nf, int flags, int act_kind,
                             float act_p0, float act_p1, const float* att, float* packed, void* stream);

/* Pack ArgMax.network (enflow/nn/argmax.py:6-10): network.0.weight [H][nf],
 * network.0.bias [H], network.2.weight [2nf][H], network.2.bias [2nf], then
 * (ABI 10) four floats [act kind, p0, p1, 0] for network.1 (ENFLOW_ACT_*; the
 * same trailing floats on every raw ArgMax vector this ABI takes: the
 * dequantiser's forward, the flow backward's dequant_raw, the standalone
 * ArgMax backward).  A non-SiLU ArgMax activation inside a flow needs
 * ENFLOW_EGCL_VARIANTS on the launches, as the EGCL variants do. */
int enflow_pack_argmax_f32(const float* raw, int hidden_nf, int node_nf,
                           float* packed, void* stream);

/*
 * LFIntegrator.forward (enflow/flow/dynamics.py:10-24), all layers fused:
 * dequantisation, then per layer the periodic neighbour list
 * (Data.edges, enflow/data/base.py:122-144), EGCL.forward
 * (enflow/nn/egcl.py:76-92) and the leapfrog update, accumulating log|detJ|.
 *   layers      : n_layers packed EGCL layers, back to back
 *                 (stride enflow_egcl_packed_size)
 *   dequant     : packed ArgMax (kind ARGMAX), ignored otherwise
 *   noise       : [num_atoms][nf]; N(0,1) draws for ARGMAX
 *                 (torch.randn in argmax.py:16), U[0,1) for FLOOR
 *   dequant_scale: Floor.dequant_scale
 *   h, g [num_atoms][nf], pos, vel [num_atoms][3] : updated in place
 *   box [num_atoms][3], r_cut [num_mols]
 *   ldj_mol [num_mols] : per-molecule log|detJ| contributions (out)
 *   ldj_total [1]      : batch log|detJ| exactly as the reference's scalar (out)
 *   pair_stats [2]     : optional (NULL = off); += unique neighbour pairs and
 *                        += reference edge-list entries, summed over layers
 *   tape               : optional (NULL = inference); training tape of
 *                        enflow_lf_tape_size floats: per layer the layer-input
 *                        state, message sums and Q, and (molecules of <= 64 atoms)
 *                        the layer's neighbour list -- pair words and per-row edge
 *                        counts, so the backward does not rebuild it -- read by
 *                        enflow_lf_backward_f32 (the layout is the library's own)
 *   pair_counts        : [n_layers][num_mols] unique pairs per layer (required
 *                        with tape)
 *   gemm_precision     : ENFLOW_PREC_* (edge_nn.2 / coord_nn.0 GEMMs)
 */
int enflow_lf_forward_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                          const int32_t* mol_ptr, const float* r_cut, const float* box,
                          float* h, float* g, float* pos, float* vel,
                          const float* layers, int n_layers,
                          int dequant_kind, const float* dequant, const float* noise,
                          float dequant_scale, float dt, float coords_weight,
                          float* ldj_mol, float* ldj_total, int32_t* err_flag,
                          uint64_t* pair_stats, float* tape, int32_t* pair_counts,
                          int gemm_precision, void* stream);

/*
 * LFIntegrator.reverse (enflow/flow/dynamics.py:26-37), all layers fused.
 * h, g, pos, vel updated in place.  With ARGMAX the final ArgMax.reverse
 * (argmax.py:27-28) is split: argmax_idx [num_atoms] (out) receives the index
 * of the first maximum and max_idx [1] (out) its batch maximum, and
 * enflow_one_hot_f32 then writes the one-hot rows (width max_idx + 1, as
 * helpers.one_hot without num_classes).  With FLOOR h is floored in place.
 */
int enflow_lf_reverse_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                          const int32_t* mol_ptr, const float* r_cut, const float* box,
                          float* h, float* g, float* pos, float* vel,
                          const float* layers, int n_layers,
                          int dequant_kind, float dt, float coords_weight,
                          int32_t* argmax_idx, int32_t* max_idx, int32_t* err_flag,
                          int gemm_precision, void* stream);

/*
 * enflow_lf_forward_f32 as one self-contained launch (the reference's
 * LFIntegrator.forward returns new tensors, dynamics.py:10-24; nothing here
 * needs a copy, a separate noise draw or a separate reduction):
 *   h_in, g_in, pos_in, vel_in : inputs, read only (NULL: the corresponding
 *                 output buffer is read, i.e. in place); outputs h, g, pos, vel
 *   noise       : the caller's draws as in enflow_lf_forward_f32, or NULL with
 *                 ARGMAX / FLOOR: drawn in the kernel, Philox4x32-10 keyed by
 *                 noise_seed, counter (atom * node_nf + q, offset noise_offset);
 *                 N(0,1) by Box-Muller for ARGMAX, U[0,1) for FLOOR.  A caller
 *                 advances noise_offset (or the seed) between calls.
 *   ticket      : device uint32, zero before the first call on it; the last
 *                 workgroup to finish reduces ldj_mol into ldj_total (same
 *                 fixed-order double sum as the separate reduction) and resets
 *                 it to zero.  One ticket per concurrently running call; NULL:
 *                 a second launch reduces, as enflow_lf_forward_f32.
 * Everything else as enflow_lf_forward_f32 (enflow_lf_forward_f32 is this call
 * with the inputs NULL, the caller's noise and no ticket).
 */
int enflow_lf_forward_io_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                             const int32_t* mol_ptr, const float* r_cut, const float* box,
                             const float* h_in, const float* g_in, const float* pos_in, const float* vel_in,
                             float* h, float* g, float* pos, float* vel,
                             const float* layers, int n_layers,
                             int dequant_kind, const float* dequant, const float* noise,
                             uint64_t noise_seed, uint64_t noise_offset,
                             float dequant_scale, float dt, float coords_weight,
                             float* ldj_mol, float* ldj_total, uint32_t* ticket, int32_t* err_flag,
                             uint64_t* pair_stats, float* tape, int32_t* pair_counts,
                             int gemm_precision, void* stream);

/* enflow_lf_reverse_f32 out of place (LFIntegrator.reverse, dynamics.py:26-37):
 * inputs h_in, g_in, pos_in, vel_in (NULL: in place), outputs h, g, pos, vel. */
int enflow_lf_reverse_io_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                             const int32_t* mol_ptr, const float* r_cut, const float* box,
                             const float* h_in, const float* g_in, const float* pos_in, const float* vel_in,
                             float* h, float* g, float* pos, float* vel,
                             const float* layers, int n_layers,
                             int dequant_kind, float dt, float coords_weight,
                             int32_t* argmax_idx, int32_t* max_idx, int32_t* err_flag,
                             int gemm_precision, void* stream);

/* ABI 12: enflow_lf_forward_io_f32 / enflow_lf_reverse_io_f32 with
 *   mol_err   (optional, [num_mols], zeroed by the caller): each molecule's own
 *             ENFLOW_ERR_* bits (err_flag keeps the OR over the batch), so a
 *             split-precision range / small-operand flag names its molecules;
 *   mol_list  (optional, [num_listed]): run only these molecules of the batch,
 *             reading and writing their atoms in place of a full launch (the
 *             same noise elements: Philox counters are keyed by the batch's
 *             atom index); the forward then reduces ldj_total over all
 *             num_mols entries of ldj_mol (ticket must be NULL).
 * The host mirror re-runs only the flagged molecules with ENFLOW_PREC_F32
 * (the reference's result) instead of the whole batch.  Molecules past
 * enflow_max_atoms() are not accepted here (-3). */
int enflow_lf_forward_io2_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                              const int32_t* mol_ptr, const float* r_cut, const float* box,
                              const float* h_in, const float* g_in, const float* pos_in, const float* vel_in,
                              float* h, float* g, float* pos, float* vel,
                              const float* layers, int n_layers,
                              int dequant_kind, const float* dequant, const float* noise,
                              uint64_t noise_seed, uint64_t noise_offset,
                              float dequant_scale, float dt, float coords_weight,
                              float* ldj_mol, float* ldj_total, uint32_t* ticket, int32_t* err_flag,
                              uint64_t* pair_stats, float* tape, int32_t* pair_counts,
                              int gemm_precision, int32_t* mol_err, const int32_t* mol_list, int num_listed,
                              void* stream);
int enflow_lf_reverse_io2_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                              const int32_t* mol_ptr, const float* r_cut, const float* box,
                              const float* h_in, const float* g_in, const float* pos_in, const float* vel_in,
                              float* h, float* g, float* pos, float* vel,
                              const float* layers, int n_layers,
                              int dequant_kind, float dt, float coords_weight,
                              int32_t* argmax_idx, int32_t* max_idx, int32_t* err_flag,
                              int gemm_precision, int32_t* mol_err, const int32_t* mol_list, int num_listed,
                              void* stream);

/* ------------------------------------------------------------------------
 * Large systems: molecules / periodic boxes with more than enflow_max_atoms()
 * atoms (e.g. the reference's example/generate.yaml, one 2944-atom LJ box).
 * Same operators, arguments and results as enflow_lf_forward_f32 /
 * enflow_lf_reverse_f32 / enflow_egcl_forward_f32 (LFIntegrator.forward /
 * .reverse, enflow/flow/dynamics.py:10-37; EGCL.forward, enflow/nn/egcl.py:76-92;
 * neighbour list enflow/data/base.py:122-144), any molecule size below 2^22
 * atoms.  Each layer runs as grid-wide launches
 * (image masks, id_mapping, pair words, one workgroup per 32-row block), so
 * `workspace` (device, enflow_lf_large_workspace_size bytes, no
 * initialisation needed) holds the per-layer neighbour list: 4 x max_mol_atoms
 * bytes per atom plus O(atoms).  Returns -6 if workspace_bytes is too small.
 *
 * Training (enflow_lf_forward_large_f32 with tape != NULL; any molecule size,
 * also 65..256-atom molecules the fused kernels run at inference): tape of
 * enflow_lf_tape_size floats (the same layout as enflow_lf_forward_f32's) and
 * pair_rows [n_layers] (out; zeroed here) = per layer the backward's pair rows
 * (sum over row blocks of the block's pair words rounded up to 32); its
 * maximum over layers is the pair_row_bound of enflow_lf_backward_large_f32.
 * ---------------------------------------------------------------------- */
int64_t enflow_lf_large_workspace_size(int num_mols, int num_atoms, int max_mol_atoms, int node_nf);

int enflow_lf_forward_large_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                                const int32_t* mol_ptr, const float* r_cut, const float* box,
                                float* h, float* g, float* pos, float* vel,
                                const float* layers, int n_layers,
                                int dequant_kind, const float* dequant, const float* noise,
                                float dequant_scale, float dt, float coords_weight,
                                float* ldj_mol, float* ldj_total, int32_t* err_flag, int gemm_precision,
                                float* tape, int32_t* pair_rows,
                                void* workspace, int64_t workspace_bytes, void* stream);

int enflow_lf_reverse_large_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                                const int32_t* mol_ptr, const float* r_cut, const float* box,
                                float* h, float* g, float* pos, float* vel,
                                const float* layers, int n_layers,
                                int dequant_kind, float dt, float coords_weight,
                                int32_t* argmax_idx, int32_t* max_idx, int32_t* err_flag,
                                int gemm_precision, void* workspace, int64_t workspace_bytes, void* stream);

int enflow_egcl_forward_large_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                                  const int32_t* mol_ptr, const float* r_cut, const float* box,
                                  const float* h, const float* pos, const float* layer,
                                  float coords_weight, float* Q, float* F, float* G,
                                  int32_t* err_flag, int gemm_precision,
                                  void* workspace, int64_t workspace_bytes, void* stream);

/* Data.edges for large systems (base.py:122-144): per row atom a, npairs[a]
 * words in pairs[a * max_mol_atoms ...], each (col << 5) | (multiplicity << 27)
 * with col the molecule-local column label; one word per column atom q with a
 * hit (a label can repeat within a row: sum the multiplicities per label). */
int enflow_neighbour_pairs_large_f32(int num_mols, int num_atoms, int max_mol_atoms, const int32_t* mol_ptr,
                                     const float* r_cut, const float* box, const float* pos,
                                     int32_t* npairs, uint32_t* pairs, int32_t* err_flag,
                                     void* workspace, int64_t workspace_bytes, void* stream);

/* helpers.one_hot (enflow/utils/helpers.py:43-52): out[num_atoms][width]. */
int enflow_one_hot_f32(const int32_t* idx, int num_atoms, int width, float* out,
                       void* stream);

/*
 * One EGCL.forward (enflow/nn/egcl.py:76-92) on Data.edges built from pos
 * (enflow/data/base.py:122-144): Q [num_atoms], F [num_atoms][3],
 * G [num_atoms][nf] (out).
 */
int enflow_egcl_forward_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                            const int32_t* mol_ptr, const float* r_cut, const float* box,
                            const float* h, const float* pos, const float* layer,
                            float coords_weight, float* Q, float* F, float* G,
                            int32_t* err_flag, void* stream);

/*
 * ArgMax.forward (enflow/nn/argmax.py:13-25): z [num_atoms][nf] (out) and
 * log_q [1] (out) with noise = the N(0,1) draw.
 */
int enflow_argmax_forward_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                              const int32_t* mol_ptr, const float* h, const float* dequant,
                              const float* noise, float* z, float* log_q_mol,
                              float* log_q, void* stream);

/*
 * Data.edges (enflow/data/base.py:122-144) as unique pairs with multiplicity:
 * pair_count[num_mols] (out) and, per molecule m, up to max_pairs entries at
 * pairs[m * max_pairs + p] = row | col << 8 | mult << 16 (molecule-local atom
 * indices, sorted by (row, col)); mult is how many times the reference's edge
 * list holds (row, col).
 */
int enflow_neighbour_pairs_f32(int num_mols, int num_atoms, int max_mol_atoms, const int32_t* mol_ptr,
                               const float* r_cut, const float* box, const float* pos,
                               int max_pairs, uint32_t* pairs, int32_t* pair_count,
                               int32_t* err_flag, void* stream);

/*
 * Alchemical_NLL.__call__ (enflow/flow/loss.py:21-24) on a flow output:
 * nll_mol [num_mols][4] (out) = {LJ energy, sum vel^2, sum h^2, sum g^2}
 * per molecule, loss [1] (out) the reference's scalar.
 */
int enflow_alchemical_nll_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf,
                              const int32_t* mol_ptr, const float* h, const float* g,
                              const float* pos, const float* vel, const float* ldj_total,
                              float kBT, float softening, float partition_func,
                              float* nll_mol, float* loss, void* stream);

/* ------------------------------------------------------------------------
 * Training (the reference's loss.backward(), enflow/main.py:219-221):
 * reverse-mode gradients of Alchemical_NLL(LFIntegrator(data)) w.r.t. every
 * EGCL / ArgMax parameter, in torch parameter layout.
 * ---------------------------------------------------------------------- */

/* Floats of the training tape enflow_lf_forward_f32 writes. */
int64_t enflow_lf_tape_size(int num_atoms, int node_nf, int hidden_nf, int n_layers);
/* ABI 12: the same for a batch whose largest molecule has max_mol_atoms atoms:
 * the tape's neighbour-list section (its tail) exists only for 33..64-atom
 * molecules, the only instance that writes and reads it; other batches' tapes
 * are that much smaller (31 % at H = 128, 57 % at H = 32, nf = 5). */
int64_t enflow_lf_tape_size_for(int num_atoms, int node_nf, int hidden_nf, int n_layers, int max_mol_atoms);

/* Backward-only packed section of one EGCL layer (transposed MFMA fragments,
 * k-contiguous node weights): size in floats, and the packing kernel (same
 * raw concatenation as enflow_pack_egcl_f32). */
int64_t enflow_egcl_bwd_packed_size(int hidden_nf, int node_nf);
int enflow_pack_egcl_bwd_f32(const float* raw, int hidden_nf, int node_nf, float* packed, void* stream);
/* ABI 13: every layer of a flow at once (default-flag SiLU layers): layer l's
 * raw concatenation at raw + l * raw_stride, written to packed + l *
 * enflow_egcl_packed_size (forward section) / enflow_egcl_bwd_packed_size
 * (backward section).  Two launches per section for the whole flow instead of
 * two per layer -- the repack after every optimiser step (enflow/main.py:
 * 217-223). */
int enflow_pack_egcl_layers_f32(const float* raw, int64_t raw_stride, int n_layers, int hidden_nf, int node_nf,
                                float* packed, void* stream);
int enflow_pack_egcl_bwd_layers_f32(const float* raw, int64_t raw_stride, int n_layers, int hidden_nf, int node_nf,
                                    float* packed, void* stream);

/* Bytes of scratch enflow_lf_backward_f32 needs.  pair_row_bound >= the sum
 * over molecules of n_m (n_m - 1) rounded up to a multiple of 32. */
int64_t enflow_lf_backward_workspace_size(int num_mols, int num_atoms, int node_nf, int hidden_nf,
                                          int n_layers, int64_t pair_row_bound);
/* The smallest workspace enflow_lf_backward_f32 accepts (two rotating
 * pair-row buffers instead of three: the layer chain then waits for the
 * weight-gradient pass two layers up, ~3 % slower at the bench batch).  The
 * backward uses three when workspace_bytes holds them. */
int64_t enflow_lf_backward_workspace_size_min(int num_mols, int num_atoms, int node_nf, int hidden_nf,
                                              int n_layers, int64_t pair_row_bound);

/*
 * Alchemical_NLL backward (enflow/flow/loss.py:11-24): adjoints of the flow
 * outputs adj_h, adj_g [num_atoms][nf], adj_pos, adj_vel [num_atoms][3] and of
 * log|detJ| adj_ldj [1] (all out), scaled by *grad_loss (NULL = 1).
 */
int enflow_alchemical_nll_backward_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf,
                                       const int32_t* mol_ptr, const float* h, const float* g,
                                       const float* pos, const float* vel, float kBT, float softening,
                                       const float* grad_loss, float* adj_h, float* adj_g, float* adj_pos,
                                       float* adj_vel, float* adj_ldj, void* stream);

/*
 * LFIntegrator.forward backward (enflow/flow/dynamics.py:10-24 with
 * enflow/nn/egcl.py:57-92 and enflow/nn/argmax.py:13-25).
 *   tape, pair_counts : written by enflow_lf_forward_f32 on the same inputs
 *   layers            : forward-packed layers (enflow_pack_egcl_f32)
 *   layers_bwd        : backward-packed layers (enflow_pack_egcl_bwd_f32)
 *   layers_raw        : raw torch-layout layers, per layer the default-flag
 *                       parameters (named_parameters order without att_nn)
 *                       followed by att_nn.0.weight [H] and att_nn.0.bias [1]
 *                       (zeros for layers without attention); stride = that
 *                       count + hidden_nf + 1
 *   dequant_raw       : raw ArgMax parameters; h_data the flow's input h
 *                       (before dequantisation) and noise its N(0,1) draw
 *   adj_h/g/pos/vel   : in: adjoints of the flow outputs; out: of the inputs
 *                       (adj_h: of the dequantised h)
 *   adj_ldj [1]       : adjoint of log|detJ|
 *   grad_layers       : out, same layout and stride as layers_raw (torch
 *                       layouts; the att_nn slots of layers without attention
 *                       are unspecified), grad_dequant: out, ArgMax layout
 *   workspace         : >= enflow_lf_backward_workspace_size bytes
 *   dequant_kind      : ENFLOW_DEQUANT_*, OR-ed with ENFLOW_EGCL_VARIANTS when
 *                       any layer carries ENFLOW_EGCL_* flags (attention,
 *                       norm_diff, tanh: all differentiated), and with
 *                       ENFLOW_BWD_F32 when the tape came from an
 *                       ENFLOW_PREC_F32 forward (the fp32-GEMM backward: the
 *                       f16x3 one recomputes the forward's activations in
 *                       f16x3, which an ENFLOW_ERR_RANGE re-run must avoid)
 */
#define ENFLOW_BWD_F32 0x200
int enflow_lf_backward_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                           const int32_t* mol_ptr, const float* r_cut, const float* box,
                           const float* tape, const int32_t* pair_counts,
                           const float* layers, const float* layers_bwd, const float* layers_raw, int n_layers,
                           int dequant_kind, const float* dequant_raw, const float* h_data, const float* noise,
                           float dt, float coords_weight,
                           float* adj_h, float* adj_g, float* adj_pos, float* adj_vel, const float* adj_ldj,
                           float* grad_layers, float* grad_dequant,
                           void* workspace, int64_t workspace_bytes, int64_t pair_row_bound,
                           int32_t* err_flag, void* stream);

/*
 * LFIntegrator.forward backward for large systems (molecules past 64 atoms;
 * the reference trains the LJ / simulated boxes of enflow/data/lj.py:32-89
 * through enflow/main.py:212-223).  Same arguments and results as
 * enflow_lf_backward_f32; tape from enflow_lf_forward_large_f32 on the same
 * inputs; pair_row_bound >= max over layers of its pair_rows (a smaller bound
 * sets ENFLOW_ERR_TOO_MANY_ATOMS and NaN-poisons the gradients).  Per layer the
 * neighbour list of the taped positions is rebuilt with the forward's kernels;
 * the column-side adjoints are summed per column in a fixed order (bitwise
 * reproducible).  Workspace: O(max_mol_atoms x atoms) + O(pair_row_bound).
 */
int64_t enflow_lf_backward_large_workspace_size(int num_mols, int num_atoms, int max_mol_atoms, int node_nf,
                                                int hidden_nf, int64_t pair_row_bound);
int enflow_lf_backward_large_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                                 const int32_t* mol_ptr, const float* r_cut, const float* box, const float* tape,
                                 const float* layers, const float* layers_bwd, const float* layers_raw, int n_layers,
                                 int dequant_kind, const float* dequant_raw, const float* h_data, const float* noise,
                                 float dt, float coords_weight,
                                 float* adj_h, float* adj_g, float* adj_pos, float* adj_vel, const float* adj_ldj,
                                 float* grad_layers, float* grad_dequant,
                                 void* workspace, int64_t workspace_bytes, int64_t pair_row_bound,
                                 int32_t* err_flag, void* stream);

/* ------------------------------------------------------------------------
 * Standalone module backward passes (the reference's EGCL and ArgMax are
 * ordinary autograd modules, enflow/nn/egcl.py:76-92, enflow/nn/argmax.py:13-25).
 * ---------------------------------------------------------------------- */

/* EGCL.forward backward: given the adjoints of its outputs adj_Q [A],
 * adj_F [A][3], adj_G [A][nf], writes adj_h [A][nf], adj_pos [A][3] (the
 * gradient reaching h and, through Edges.coord_diff, the positions) and
 * grad_layer (one layer in the layers_raw layout of enflow_lf_backward_f32).
 * tape / pair_counts: written by a one-layer enflow_lf_forward_f32 on the same
 * h / pos (dequant NONE, dt 0); layer / layer_bwd / layer_raw: that layer
 * packed; egcl_flags: its ENFLOW_EGCL_* flags (| ENFLOW_BWD_F32: the tape is from an
 * ENFLOW_PREC_F32 forward).  Molecules of <= 64 atoms. */
int64_t enflow_egcl_backward_workspace_size(int num_mols, int num_atoms, int node_nf, int hidden_nf,
                                            int64_t pair_row_bound);
int enflow_egcl_backward_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                             const int32_t* mol_ptr, const float* r_cut, const float* box,
                             const float* tape, const int32_t* pair_counts,
                             const float* layer, const float* layer_bwd, const float* layer_raw, int egcl_flags,
                             float coords_weight, const float* adj_Q, const float* adj_F, const float* adj_G,
                             float* adj_h, float* adj_pos, float* grad_layer,
                             void* workspace, int64_t workspace_bytes, int64_t pair_row_bound,
                             int32_t* err_flag, void* stream);

/* The same for molecules past 64 atoms: tape / pair_rows from a one-layer
 * enflow_lf_forward_large_f32 on the same h / pos (dequant NONE, dt 0; its
 * pair_rows[0] = the pair_row_bound), then the large-system backward. */
int64_t enflow_egcl_backward_large_workspace_size(int num_mols, int num_atoms, int max_mol_atoms, int node_nf,
                                                  int hidden_nf, int64_t pair_row_bound);
int enflow_egcl_backward_large_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                                   const int32_t* mol_ptr, const float* r_cut, const float* box, const float* tape,
                                   const float* layer, const float* layer_bwd, const float* layer_raw,
                                   int egcl_flags, float coords_weight, const float* adj_Q, const float* adj_F,
                                   const float* adj_G, float* adj_h, float* adj_pos, float* grad_layer,
                                   void* workspace, int64_t workspace_bytes, int64_t pair_row_bound,
                                   int32_t* err_flag, void* stream);

/* ArgMax.forward backward: adjoints of z [A][nf] and of log_q [1] -> the
 * gradient of ArgMax.network's parameters (grad_dequant, raw layout of
 * enflow_pack_argmax_f32).  noise: the forward's N(0,1) draw; h: its input.
 * mol_ptr chunks the atoms (<= 64 per chunk; ArgMax is per atom). */
int64_t enflow_argmax_backward_workspace_size(int num_atoms, int node_nf, int hidden_nf);
int enflow_argmax_backward_f32(int num_mols, int num_atoms, int max_mol_atoms, int node_nf, int hidden_nf,
                               const int32_t* mol_ptr, const float* h, const float* dequant_raw, const float* noise,
                               const float* adj_z, const float* adj_log_q, float* grad_dequant,
                               void* workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Per-kernel timing (measurement only; no reference counterpart).  When
 * enabled, every kernel this library launches is bracketed by a hipEvent pair
 * on its own launch stream; collect() waits for the recorded events and adds
 * their elapsed times per kernel name.  Off by default (no events recorded).
 * ---------------------------------------------------------------------- */
int enflow_timing_enable(int on);
/* Wait for and accumulate the recorded events; returns the number of names. */
int enflow_timing_collect(void);
/* Entry i: kernel name (NUL-terminated, truncated to name_len), total
 * milliseconds and launch count since the last reset.  -1 if i is out of range. */
int enflow_timing_entry(int i, char* name, int name_len, double* total_ms, int64_t* launches);
int enflow_timing_reset(void);

#ifdef __cplusplus
}
#endif

#endif /* ENFLOW_HIP_H */
