// ordering.cpp -- nested-dissection order of the pose graph (specification in ordering.hpp).
#include "ordering.hpp"

#include <algorithm>
#include <cstdlib>
#include <thread>

namespace orbgpu {

namespace {

constexpr int kParDepth = 2;    // the top two dissection levels split over host threads
constexpr int kParMin = 256;     // ... when both sides have this many poses

struct Nd {
    const std::vector<int>& as;
    const std::vector<int>& adj;
    int leaf;
    NdTree* t;
    std::vector<int> inS;    // stamp: node is in the current set
    std::vector<int> mark;   // stamp: visited by the current BFS
    int stamp = 0;

    // BFS level sets from r over the nodes with inS == sid
    void levels(int r, int sid, std::vector<std::vector<int>>& L) {
        L.clear();
        const int st = ++stamp;
        mark[r] = st;
        L.push_back({r});
        for (;;) {
            std::vector<int> nxt;
            for (int v : L.back())
                for (int e = as[v]; e < as[v + 1]; e++) {
                    const int w = adj[e];
                    if (inS[w] == sid && mark[w] != st) {
                        mark[w] = st;
                        nxt.push_back(w);
                    }
                }
            if (nxt.empty()) break;
            std::sort(nxt.begin(), nxt.end());
            L.push_back(std::move(nxt));
        }
    }

    int new_node(int s, int e, int h) {
        t->start.push_back(s);
        t->end.push_back(e);
        t->parent.push_back(-1);
        t->height.push_back(h);
        return (int)t->start.size() - 1;
    }

    // appends the roots of S's subtrees to `roots`
    void order(std::vector<int> S, std::vector<int>& roots, int depth = 0) {
        const int sid = ++stamp;
        for (int v : S) inS[v] = sid;
        const int n = (int)S.size();
        // the level sets from S[0] reach all of S exactly when S is connected: the usual case,
        // and then the component search below (the same traversal) is skipped
        std::vector<std::vector<int>> L;
        if (n > leaf) {
            levels(S[0], sid, L);
            size_t reach = 0;
            for (const auto& lv : L) reach += lv.size();
            if ((int)reach != n) L.clear();
        }
        // connected components, in order of their smallest node
        if (L.empty()) {
            std::vector<std::vector<int>> comps;
            const int st = ++stamp;
            for (int s0 : S) {
                if (mark[s0] == st) continue;
                std::vector<int> comp{s0}, q{s0};
                mark[s0] = st;
                for (size_t h = 0; h < q.size(); h++) {
                    const int v = q[h];
                    for (int e = as[v]; e < as[v + 1]; e++) {
                        const int w = adj[e];
                        if (inS[w] == sid && mark[w] != st) {
                            mark[w] = st;
                            q.push_back(w);
                            comp.push_back(w);
                        }
                    }
                }
                std::sort(comp.begin(), comp.end());
                comps.push_back(std::move(comp));
            }
            if (comps.size() > 1) {
                for (auto& c : comps) order(std::move(c), roots, depth);
                return;
            }
        }
        auto make_leaf = [&]() {
            const int s = (int)t->perm.size();
            t->perm.insert(t->perm.end(), S.begin(), S.end());
            roots.push_back(new_node(s, (int)t->perm.size(), 0));
        };
        if (n <= leaf) return make_leaf();
        if (L.empty()) levels(S[0], sid, L);
        const int u = L.back()[0];
        levels(u, sid, L);
        const int h = (int)L.size() - 1;
        if (h < 2) return make_leaf();
        int best = -1;
        long long bk[4] = {0, 0, 0, 0};
        int A = 0;
        for (int m = 1; m < h; m++) {
            A += (int)L[m - 1].size();
            const int Lm = (int)L[m].size(), B = n - A - Lm;
            const bool ok = 5LL * std::min(A, B) >= n;
            const long long key[4] = {ok ? 0 : 1, ok ? Lm : std::abs(A - B), std::abs(A - B), m};
            if (best < 0 || std::lexicographical_compare(key, key + 4, bk, bk + 4)) {
                best = m;
                std::copy(key, key + 4, bk);
            }
        }
        std::vector<int> Aset, Bset;
        for (int i = 0; i < best; i++) Aset.insert(Aset.end(), L[i].begin(), L[i].end());
        for (int i = best + 1; i <= h; i++) Bset.insert(Bset.end(), L[i].begin(), L[i].end());
        std::sort(Aset.begin(), Aset.end());
        std::sort(Bset.begin(), Bset.end());
        std::vector<int> sep = std::move(L[best]);
        std::vector<int> kids;
        if (depth < kParDepth && (int)Aset.size() >= kParMin && (int)Bset.size() >= kParMin) {
            // the two sides are independent: B on a thread of its own into a tree fragment (own
            // stamps), spliced after A's nodes -- the same tree as the sequential recursion
            NdTree tb;
            std::vector<int> kidsB;
            Nd nb{as, adj, leaf, &tb, std::vector<int>(inS.size(), 0), std::vector<int>(mark.size(), 0)};
            std::thread th([&] { nb.order(std::move(Bset), kidsB, depth + 1); });
            order(std::move(Aset), kids, depth + 1);
            th.join();
            const int basePerm = (int)t->perm.size(), baseNode = (int)t->start.size();
            t->perm.insert(t->perm.end(), tb.perm.begin(), tb.perm.end());
            for (size_t k = 0; k < tb.start.size(); k++) {
                t->start.push_back(tb.start[k] + basePerm);
                t->end.push_back(tb.end[k] + basePerm);
                t->parent.push_back(tb.parent[k] >= 0 ? tb.parent[k] + baseNode : -1);
                t->height.push_back(tb.height[k]);
            }
            for (int c : kidsB) kids.push_back(c + baseNode);
        } else {
            order(std::move(Aset), kids, depth + 1);
            order(std::move(Bset), kids, depth + 1);
        }
        int hmax = 0;
        for (int c : kids) hmax = std::max(hmax, t->height[c]);
        const int s = (int)t->perm.size();
        t->perm.insert(t->perm.end(), sep.begin(), sep.end());
        const int id = new_node(s, (int)t->perm.size(), hmax + 1);
        for (int c : kids) t->parent[c] = id;
        roots.push_back(id);
    }
};

}  // namespace

void nd_order(int n, const std::vector<int>& adjStart, const std::vector<int>& adj, int leaf, NdTree* out) {
    *out = NdTree{};
    if (n <= 0) return;
    Nd nd{adjStart, adj, leaf, out, std::vector<int>(n, 0), std::vector<int>(n, 0)};
    std::vector<int> all(n), roots;
    for (int i = 0; i < n; i++) all[i] = i;
    nd.order(std::move(all), roots);
}

void nd_assign(const NdTree& t, int R, std::vector<int>* owner) {
    const int nn = (int)t.start.size();
    owner->assign(nn, R <= 1 ? 0 : -1);
    if (R <= 1 || nn == 0) return;
    // subtree pose counts (children precede their parent in postorder)
    std::vector<long long> cost(nn, 0);
    std::vector<std::vector<int>> kids(nn);
    for (int k = 0; k < nn; k++) {
        cost[k] += t.end[k] - t.start[k];
        if (t.parent[k] >= 0) {
            cost[t.parent[k]] += cost[k];
            kids[t.parent[k]].push_back(k);
        }
    }
    // longest-processing-time assignment of a frontier; its makespan in poses
    auto lpt = [&](std::vector<int> f, std::vector<int>* rootOwner) {
        std::sort(f.begin(), f.end(), [&](int a, int b) { return cost[a] != cost[b] ? cost[a] > cost[b] : a < b; });
        std::vector<long long> load(R, 0);
        for (int k : f) {
            int r = 0;
            for (int q = 1; q < R; q++)
                if (load[q] < load[r]) r = q;
            if (rootOwner) (*rootOwner)[k] = r;
            load[r] += cost[k];
        }
        return *std::max_element(load.begin(), load.end());
    };
    // split the largest splittable subtree again and again (its root joins the separators every
    // rank factors), up to 4R subtrees; keep the frontier of the step with the least (separator
    // poses + the most poses one rank gets) -- one split can raise that sum while the next ones
    // lower it, so every prefix of the split sequence is scored
    std::vector<int> front;
    for (int k = 0; k < nn; k++)
        if (t.parent[k] < 0) front.push_back(k);
    long long shared = 0, bestT = lpt(front, nullptr);
    std::vector<int> bestFront = front;
    while ((int)front.size() < 4 * R) {
        int pick = -1;
        for (int q = 0; q < (int)front.size(); q++) {
            const int k = front[q];
            if (kids[k].empty()) continue;
            if (pick < 0 || cost[k] > cost[front[pick]] || (cost[k] == cost[front[pick]] && k < front[pick])) pick = q;
        }
        if (pick < 0) break;
        const int k = front[pick];
        front.erase(front.begin() + pick);
        front.insert(front.end(), kids[k].begin(), kids[k].end());
        shared += t.end[k] - t.start[k];
        const long long T = shared + lpt(front, nullptr);
        if (T < bestT) {
            bestT = T;
            bestFront = front;
        }
    }
    front = bestFront;
    std::vector<int> rootOwner(nn, -1);
    lpt(front, &rootOwner);
    // a subtree's nodes take its root's rank: parents follow their children in postorder, so
    // descending indices visit a parent first
    for (int k = nn - 1; k >= 0; k--) {
        if (rootOwner[k] >= 0) (*owner)[k] = rootOwner[k];
        else if (t.parent[k] >= 0 && (*owner)[t.parent[k]] >= 0) (*owner)[k] = (*owner)[t.parent[k]];
    }
}

}  // namespace orbgpu
