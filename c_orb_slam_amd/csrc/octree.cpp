// octree.cpp -- see octree.hpp.  Reference: src/ORBextractor.cc:481-763.
#include "octree.hpp"

#include <algorithm>
#include <cmath>

namespace orbgpu {

int OctreeWorker::new_node(int x0, int y0, int x1, int y1) {
    Node n;
    n.x0 = x0; n.y0 = y0; n.x1 = x1; n.y1 = y1;
    n.kbeg = 0; n.kcnt = 0; n.prev = n.next = -1; n.seq = 0; n.noMore = false;
    nodes_.push_back(n);
    return (int)nodes_.size() - 1;
}

void OctreeWorker::push_front(int idx) {
    Node& n = nodes_[idx];
    n.prev = -1;
    n.next = head_;
    if (head_ >= 0) nodes_[head_].prev = idx;
    head_ = idx;
    n.seq = seq_++;
    size_++;
}

int OctreeWorker::erase(int idx) {
    Node& n = nodes_[idx];
    const int nx = n.next;
    if (n.prev >= 0) nodes_[n.prev].next = n.next; else head_ = n.next;
    if (n.next >= 0) nodes_[n.next].prev = n.prev;
    size_--;
    return nx;
}

// ExtractorNode::DivideNode, ORBextractor.cc:481-537.  Children are rectangles
// n1=(UL..), n2, n3, n4; keys keep their order inside each child.
void OctreeWorker::divide(int pidx, const OctKey* keys, int ch[4]) {
    const Node p = nodes_[pidx];
    const int halfX = (int)std::ceil((float)(p.x1 - p.x0) / 2);
    const int halfY = (int)std::ceil((float)(p.y1 - p.y0) / 2);
    const int mx = p.x0 + halfX, my = p.y0 + halfY;
    ch[0] = new_node(p.x0, p.y0, mx, my);
    ch[1] = new_node(mx, p.y0, p.x1, my);
    ch[2] = new_node(p.x0, my, mx, p.y1);
    ch[3] = new_node(mx, my, p.x1, p.y1);
    int cnt[4] = {0, 0, 0, 0};
    tmp_.resize(p.kcnt);
    const float fmx = (float)mx, fmy = (float)my;
    for (int i = 0; i < p.kcnt; i++) {
        const OctKey& k = keys[arena_[p.kbeg + i]];
        const int d = (k.x < fmx) ? (k.y < fmy ? 0 : 2) : (k.y < fmy ? 1 : 3);
        tmp_[i] = d;
        cnt[d]++;
    }
    int base = (int)arena_.size();
    arena_.resize(base + p.kcnt);
    int pos[4];
    pos[0] = base; pos[1] = pos[0] + cnt[0]; pos[2] = pos[1] + cnt[1]; pos[3] = pos[2] + cnt[2];
    for (int c = 0; c < 4; c++) {
        nodes_[ch[c]].kbeg = pos[c];
        nodes_[ch[c]].kcnt = cnt[c];
        nodes_[ch[c]].noMore = cnt[c] == 1;
    }
    const int pb = p.kbeg;
    for (int i = 0; i < p.kcnt; i++) arena_[pos[tmp_[i]]++] = arena_[pb + i];
}

int OctreeWorker::distribute(const OctKey* keys, int nkeys, int minX, int maxX, int minY, int maxY,
                             int N, std::vector<uint32_t>& out) {
    out.clear();
    nodes_.clear();
    arena_.clear();
    head_ = -1; size_ = 0; seq_ = 0;
    const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
    if (nIni <= 0) return -1;
    const float hX = (float)(maxX - minX) / nIni;

    // initial nodes (push_back order)
    std::vector<int> ini(nIni);
    int tail = -1;
    for (int i = 0; i < nIni; i++) {
        int id = new_node((int)(hX * (float)i), 0, (int)(hX * (float)(i + 1)), maxY - minY);
        Node& n = nodes_[id];
        n.prev = tail; n.next = -1;
        if (tail >= 0) nodes_[tail].next = id; else head_ = id;
        tail = id;
        n.seq = seq_++;
        size_++;
        ini[i] = id;
    }
    // counting sort of keys into initial nodes, order kept
    std::vector<int> cnt(nIni + 1, 0);
    tmp_.resize(nkeys);
    for (int i = 0; i < nkeys; i++) {
        int b = (int)(size_t)(keys[i].x / hX);
        tmp_[i] = b;
        cnt[b + 1]++;
    }
    for (int i = 0; i < nIni; i++) cnt[i + 1] += cnt[i];
    arena_.resize(nkeys);
    for (int i = 0; i < nIni; i++) { nodes_[ini[i]].kbeg = cnt[i]; nodes_[ini[i]].kcnt = cnt[i + 1] - cnt[i]; }
    {
        std::vector<int> pos(cnt.begin(), cnt.end() - 1);
        for (int i = 0; i < nkeys; i++) arena_[pos[tmp_[i]]++] = i;
    }
    for (int lit = head_; lit >= 0;) {
        Node& n = nodes_[lit];
        if (n.kcnt == 1) { n.noMore = true; lit = n.next; }
        else if (n.kcnt == 0) lit = erase(lit);
        else lit = n.next;
    }

    bool bFinish = false;
    while (!bFinish) {
        int prevSize = size_;
        int nToExpand = 0;
        vs_.clear();
        for (int lit = head_; lit >= 0;) {
            if (nodes_[lit].noMore) { lit = nodes_[lit].next; continue; }
            int ch[4];
            divide(lit, keys, ch);
            for (int c = 0; c < 4; c++) {
                if (nodes_[ch[c]].kcnt > 0) {
                    push_front(ch[c]);
                    if (nodes_[ch[c]].kcnt > 1) {
                        nToExpand++;
                        vs_.push_back({nodes_[ch[c]].kcnt, nodes_[ch[c]].seq, ch[c]});
                    }
                }
            }
            lit = erase(lit);
        }
        if (size_ >= N || size_ == prevSize) {
            bFinish = true;
        } else if (size_ + nToExpand * 3 > N) {
            while (!bFinish) {
                prevSize = size_;
                prev_ = vs_;
                vs_.clear();
                std::sort(prev_.begin(), prev_.end(), [](const SizePtr& a, const SizePtr& b) {
                    return a.n != b.n ? a.n < b.n : a.seq < b.seq;
                });
                for (int j = (int)prev_.size() - 1; j >= 0; j--) {
                    int ch[4];
                    divide(prev_[j].idx, keys, ch);
                    for (int c = 0; c < 4; c++) {
                        if (nodes_[ch[c]].kcnt > 0) {
                            push_front(ch[c]);
                            if (nodes_[ch[c]].kcnt > 1)
                                vs_.push_back({nodes_[ch[c]].kcnt, nodes_[ch[c]].seq, ch[c]});
                        }
                    }
                    erase(prev_[j].idx);
                    if (size_ >= N) break;
                }
                if (size_ >= N || size_ == prevSize) bFinish = true;
            }
        }
    }
    // retain the max-response key of each node (first wins ties), list order
    for (int lit = head_; lit >= 0; lit = nodes_[lit].next) {
        const Node& n = nodes_[lit];
        int best = arena_[n.kbeg];
        float maxResp = keys[best].response;
        for (int k = 1; k < n.kcnt; k++) {
            int id = arena_[n.kbeg + k];
            if (keys[id].response > maxResp) { best = id; maxResp = keys[id].response; }
        }
        out.push_back(keys[best].packed);
    }
    return (int)out.size();
}

}  // namespace orbgpu
