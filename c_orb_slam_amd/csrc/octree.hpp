// octree.hpp -- host-side DistributeOctTree for the extractor pipeline.
//
// Reference: ORBextractor::DistributeOctTree + ExtractorNode::DivideNode,
// src/ORBextractor.cc:481-763.  The algorithm is order-defining (std::list
// push_front order, first-max ties) and cheap (~10^4 keys per image), so it
// stays on the host between the GPU FAST/compaction kernels and the GPU
// orientation/rBRIEF kernel.  This is an arena/index restatement of the
// std::list version: nodes are axis-aligned rectangles (x0,y0,x1,y1), each
// node's keys a contiguous slice of an arena, the list an index-linked list.
//
// The reference's phase-2 `sort(vector<pair<int,ExtractorNode*>>)` breaks
// size ties by heap address; we break them by node creation order (the
// address order of a fresh heap) -- DESIGN.md, Appendix quirk Q1.
#pragma once
#include <cstdint>
#include <vector>

namespace orbgpu {

struct OctKey {
    float x, y;       // relative to (minBorderX, minBorderY)
    float response;
    uint32_t packed;  // caller payload, returned for the selected keys
};

class OctreeWorker {
public:
    // Returns the number of selected keys written to `out` (list order).
    int distribute(const OctKey* keys, int nkeys, int minX, int maxX, int minY, int maxY, int N,
                   std::vector<uint32_t>& out);

private:
    struct Node {
        int x0, y0, x1, y1;
        int kbeg, kcnt;   // slice of arena_
        int prev, next;
        long seq;
        bool noMore;
    };
    std::vector<Node> nodes_;
    std::vector<int> arena_;
    std::vector<int> tmp_;
    struct SizePtr { int n; long seq; int idx; };
    std::vector<SizePtr> vs_, prev_;
    int head_ = -1, size_ = 0;
    long seq_ = 0;

    int new_node(int x0, int y0, int x1, int y1);
    void push_front(int idx);
    int erase(int idx);
    void divide(int pidx, const OctKey* keys, int ch[4]);
};

}  // namespace orbgpu
