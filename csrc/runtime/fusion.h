// Planner fusion of elementwise regions into one generated kernel.
//
// A region is a connected set of elementwise ops (unary, binary with numpy
// broadcasting, Cast), metadata views (ExpandDims / Squeeze / unit-dim
// Reshape / Identity) and broadcasts (Tile of unit dims, BroadcastTo) whose
// intermediate values have no consumer outside the region. It is evaluated by
// ONE kernel that reads each external input (leaf) once per output element
// through a stride map (0 on broadcast dims) and writes only the region's
// root: no intermediate (and no tiled copy) is materialised in HBM.
//
// Example (reference K-Means distance graph,
// src/main/python/tensorframes_snippets/kmeans_demo.py:31-42):
//   t1 = tile(expand_dims(center_squares, 0), [n, 1])
//   t2 = tile(expand_dims(squares, 1), [1, k])
//   distances = t1 + t2 - 2 * prods
// becomes one kernel over [n, k] with leaves center_squares (stride [0, 1]),
// squares (stride [1, 0]), 2 (scalar) and prods (linear).
//
// The kernel source is generated per region signature (dtypes, expression,
// leaf access kinds, index width) and compiled at plan time by runtime/jit.*.
#pragma once

#include <map>
#include <set>
#include <string>
#include <vector>

#include "../ir/graph.h"

namespace tfa {

struct FusedLeaf {
  TensorRef ref;                 // external tensor read by the region
  DType dtype = DType::INVALID;
  int kind = 0;                  // 0 linear (same layout as the output), 1 scalar, 2 strided
  std::vector<int64_t> coef;     // element stride per collapsed output dim (kind 2)
};

struct FusedRegion {
  // kind 0: elementwise region, writes its root's value over the root shape.
  // kind 1: row reduction: one or more sibling reductions (Sum/Mean/Min/Max/
  //         Prod/ArgMin/ArgMax over the same trailing axes of the same tensor X)
  //         in one pass, X computed on the fly by the region (the prologue)
  //         or read directly (no prologue). X is viewed as [outer, inner].
  int kind = 0;
  int root = -1;                 // node whose output 0 the region computes (-1: X is a plain leaf)
  std::vector<int> nodes;        // member (prologue) nodes, topological order
  std::vector<int> outputs;      // nodes whose output 0 the kernel writes (kind 0: {root})
  std::vector<std::string> red_ops;  // kind 1: per output
  std::vector<FusedLeaf> leaves;
  std::vector<int64_t> dims;     // collapsed dims of the evaluated index space
  int outer_rank = 0;            // kind 1: the first outer_rank collapsed dims index rows
  int64_t numel = 0;             // elements evaluated (kind 1: outer * inner)
  int64_t outer = 0, inner = 0;  // kind 1
  DType out_dtype = DType::INVALID;
  int compute_ops = 0;           // non-view ops evaluated per element
  std::string source;            // generated HIP source
  std::string entry;             // kernel name
  std::string expr;              // readable expression (describe)
  int block = 256;
  int64_t grid = 1;
};

struct FusionInput {
  const Graph* g;
  const Graph::Infos* infos;
  std::vector<int> runtime;                 // runtime nodes, topological order
  std::set<int> excluded;                   // nodes already claimed (GEMM epilogues, ...)
  std::set<TensorRef> fetched;
  std::map<int, std::vector<int>> consumers;  // node -> runtime consumer nodes (with multiplicity)
};

// Regions of a GPU plan: row reductions first (claiming their prologues),
// then elementwise regions (each has >= 2 compute ops, or materialises a
// broadcast).
std::vector<FusedRegion> find_fused_regions(const FusionInput& in);

// Kernel argument block of a region for concrete leaf/output pointers.
std::vector<int64_t> fused_args(const FusedRegion& r, const std::vector<const void*>& leaf_ptrs,
                                const std::vector<void*>& outs);

// Launch geometry of elementwise regions.
constexpr int kFusedBlock = 256;
constexpr int kFusedEPT = 4;  // elements per thread

// Disable with TFA_FUSION=0.
bool fusion_enabled();
// the op can be evaluated inside a fused elementwise region (no HBM value)
bool fusible_op(const std::string& op);

}  // namespace tfa
