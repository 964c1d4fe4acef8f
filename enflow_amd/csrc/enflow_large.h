// enflow_large.h -- shared between the large-system forward (enflow_large.hip)
// and its training backward (enflow_backward.hip): the per-layer argument block,
// the workspace layout and the neighbour-search launch sequence.
#ifndef ENFLOW_LARGE_H
#define ENFLOW_LARGE_H
#include "flow_device.h"

struct LgArgs {
  const int32_t* mol_ptr;
  const float* r_cut;
  const float* box;
  float* h;          // this layer's state (forward: read only here, next state -> h2 / pos2)
  float* g;
  float* pos;
  float* vel;
  float* h2;
  float* pos2;
  const float* layer;   // packed EGCL layer
  int nf;
  float dt, cw;
  uint32_t* mask;       // [A]
  int32_t* idmap;       // [A] molecule-local labels (-1 past the surviving images)
  int32_t* npairs;      // [A] pair words of row a
  int32_t* cntrow;      // [A] edges of row a (with multiplicity)
  uint32_t* pairs;      // [A][max_n]
  int max_n;
  int32_t* blk_start;   // [M + 1] first row block of molecule m
  float* aabb;          // [M][6] bounding box of the molecule's positions (this layer)
  int rbl;              // rows per block (4 .. 32; the host picks it to fill the CUs)
  float* ldj_blk;       // [blocks] log|detJ| per row block
  float* Qo;            // EGCL mode outputs (else null)
  float* Fo;
  float* Go;
  int32_t* err;
  int num_mols, num_atoms;
  // training (enflow_lf_forward_large_f32 with a tape; enflow_lf_backward_large_f32)
  float* tape;          // forward: the layer-input state, message sums and Q of every layer
  int layer_idx, n_layers;
  int32_t* pair_rows;   // forward: [n_layers] += the 32-aligned pair words of every row block
  int32_t* smap;        // [A][max_n] slot of column q in row a's words (-1: no hit), or null
};

// largest m with ptr[m] <= x (ptr non-decreasing, ptr[0] = 0 <= x < ptr[count])
__device__ __forceinline__ int seg_of(const int32_t* __restrict__ ptr, int count, int x) {
  int lo = 0, hi = count;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (ptr[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

struct LgWorkspace { size_t mask, idmap, npairs, cntrow, blk_start, aabb, ldj_blk, pos2, h2, pairs, total; };
static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
LgWorkspace lg_workspace(int num_mols, int num_atoms, int max_n, int nf);
int lg_rows(int num_atoms);
LgArgs lg_args(int num_mols, int num_atoms, int max_n, int nf, const int32_t* mol_ptr, const float* r_cut,
               const float* box, float* h, float* g, float* pos, float* vel, float dt, float cw,
               int32_t* err, void* ws);
// row blocks (blk_start) of B.rbl rows per molecule
void lg_setup(hipStream_t st, const LgArgs& B);
// the neighbour list of B.pos: image masks, id_mapping, pair words (+ B.smap)
void lg_search(hipStream_t st, const LgArgs& B);
// an upper bound of the number of row blocks (grid size of the per-block kernels)
static inline int lg_grid(const LgArgs& B) { return B.num_atoms / B.rbl + B.num_mols + 1; }

#endif
