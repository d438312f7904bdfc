// ordering.hpp -- fill-reducing elimination order of the reduced pose system (host).
//
// The reference factors the Schur complement with Eigen's SimplicialLDLT after an AMD
// ordering computed once per structure (Thirdparty/g2o/g2o/solvers/linear_solver_eigen.h:
// 60-124).  Here the order is a nested dissection of the pose graph (poses adjacent when they
// share a map point), for two reasons: the fill stays bounded on the long-range covisibility
// of a loop-closed map (natural order fills the whole envelope between the two ends of a
// loop), and the separator tree is the task tree of the GPU factorisation -- the subtrees
// under a separator share no pose, so they are factored by concurrent workgroups (ldlt.hip).
//
// The order is a pure function of the graph (integer arithmetic, sorted sets, no hashing), so
// every rank of a sharded BA and the CPU oracle (oracle/ordering.c, the same specification)
// derive the same permutation:
//   order(S)  S = sorted node set
//     components of S (BFS from the smallest unvisited node, in ascending order of their
//       smallest node): more than one -> order(C) for each, no separator;
//     |S| <= leaf -> a leaf: S in ascending order;
//     else BFS level sets from r = S[0]; u = the smallest node of the last level; level sets
//       L_0..L_h from u (each sorted).  h < 2 -> a leaf.  Separator L_m, m in [1, h-1],
//       minimising (ok ? 0 : 1, ok ? |L_m| : |A-B|, |A-B|, m) with A = |L_0..L_m-1|,
//       B = |S| - A - |L_m|, ok = 5 min(A, B) >= |S|;
//     order(L_0 u .. u L_m-1), order(L_m+1 u .. u L_h), then L_m (ascending): postorder.
#pragma once
#include <vector>

namespace orbgpu {

constexpr int kNdLeafPoses = 32;   // leaf size of the pose systems' nested dissection (ldlt.hip, partitioner)

struct NdTree {
    std::vector<int> perm;      // perm[k] = node (pose) at elimination position k
    // tree nodes in postorder: positions [start, end) of perm, parent (-1 = root), height
    // (0 = leaf, else 1 + max over children)
    std::vector<int> start, end, parent, height;
};

// adjStart (n + 1) / adj: symmetric adjacency, each list sorted ascending, no self loops.
void nd_order(int n, const std::vector<int>& adjStart, const std::vector<int>& adj, int leaf, NdTree* out);

// Ranks of a sharded factorisation over the separator tree: owner[k] = the rank that factors
// node k alone (a whole subtree per rank), -1 = a separator above the ranks' subtrees, factored
// by every rank.  The largest splittable subtree (in poses) is split again and again -- its
// root joins the separators -- up to 4R subtrees, and the step with the least (separator poses +
// the most poses one rank gets) is kept; the subtrees go to ranks by longest-processing-time
// first.  A pure function of the tree: every rank and the point partitioner derive the same
// assignment.
void nd_assign(const NdTree& t, int R, std::vector<int>* owner);

}  // namespace orbgpu
