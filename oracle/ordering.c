/*
 * ordering.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * Elimination order and block-sparse LDL^T of the reduced pose system for large bundle
 * adjustments.  The reference factors the Schur complement with Eigen's SimplicialLDLT after
 * an AMD ordering computed once per structure (Thirdparty/g2o/g2o/solvers/
 * linear_solver_eigen.h:60-124).  Eigen is not in this image and AMD's tie rules are not
 * pinned by any reference fixture, so the oracle follows the product's canonical choice: a
 * nested dissection of the pose graph (c_orb_slam_amd/csrc/ordering.hpp states it).  The
 * specification, restated here independently:
 *   order(S)  S = sorted node set
 *     components of S (BFS from the smallest unvisited node, in ascending order of their
 *       smallest node): more than one -> order(C) for each;
 *     |S| <= leaf -> S ascending;
 *     else BFS level sets from S[0]; u = the smallest node of the last level; level sets
 *       L_0..L_h from u (each sorted).  h < 2 -> S ascending.  Separator L_m, m in [1, h-1],
 *       minimising (ok ? 0 : 1, ok ? |L_m| : |A-B|, |A-B|, m), A = |L_0..L_m-1|,
 *       B = |S| - A - |L_m|, ok = 5 min(A, B) >= |S|;
 *     order(L_0..L_m-1), order(L_m+1..L_h), then L_m ascending.
 * The factorisation is a right-looking LDL^T on the permuted upper triangle stored as the
 * nonzero (group x group) blocks of its symbolic fill.  Per element it performs the dense
 * routine's operation sequence (ora_ldlt_solve): updates from every pivot k in ascending k,
 * l == 0 skipped; forward y_i -= L[i][k] y_k (k ascending), y /= d, backward k descending --
 * the sequence the GPU's tiled, level-scheduled factorisation performs.
 */
#include "orb_oracle.h"
#include <stdlib.h>
#include <string.h>

static int cmp_int(const void* a, const void* b)
{
    const int x = *(const int*)a, y = *(const int*)b;
    return x < y ? -1 : x > y;
}

typedef struct {
    const int* as;
    const int* adj;
    int leaf;
    int* inS;
    int* mark;
    int stamp;
    int* perm;
    int np;
} nd_ctx;

/* BFS level sets from r over nodes with inS == sid: nodes in `lv` (level by level, each level
 * sorted), level k = lv[ls[k] .. ls[k+1]); returns the number of levels */
static int nd_levels(nd_ctx* c, int r, int sid, int* lv, int* ls)
{
    const int st = ++c->stamp;
    int n = 0, h = 0;
    c->mark[r] = st;
    lv[n++] = r;
    ls[0] = 0;
    ls[1] = 1;
    for (;;) {
        const int a = ls[h], b = ls[h + 1];
        for (int t = a; t < b; t++) {
            const int v = lv[t];
            for (int e = c->as[v]; e < c->as[v + 1]; e++) {
                const int w = c->adj[e];
                if (c->inS[w] == sid && c->mark[w] != st) {
                    c->mark[w] = st;
                    lv[n++] = w;
                }
            }
        }
        if (n == b) break;
        qsort(lv + b, n - b, sizeof(int), cmp_int);
        h++;
        ls[h + 1] = n;
    }
    return h + 1;
}

static void nd_order_set(nd_ctx* c, int* S, int n)
{
    if (n <= 0 || n > (1 << 28)) return;
    const int sid = ++c->stamp;
    for (int i = 0; i < n; i++) c->inS[S[i]] = sid;
    /* connected components, in order of their smallest node */
    {
        int* comp = (int*)malloc(sizeof(int) * n);
        int* cs = (int*)malloc(sizeof(int) * (n + 1));
        int nc = 0, m = 0;
        const int st = ++c->stamp;
        for (int i = 0; i < n; i++) {
            const int s0 = S[i];
            if (c->mark[s0] == st) continue;
            cs[nc++] = m;
            int h = m;
            comp[m++] = s0;
            c->mark[s0] = st;
            for (; h < m; h++) {
                const int v = comp[h];
                for (int e = c->as[v]; e < c->as[v + 1]; e++) {
                    const int w = c->adj[e];
                    if (c->inS[w] == sid && c->mark[w] != st) {
                        c->mark[w] = st;
                        comp[m++] = w;
                    }
                }
            }
        }
        cs[nc] = m;
        if (nc > 1) {
            for (int k = 0; k < nc; k++) qsort(comp + cs[k], cs[k + 1] - cs[k], sizeof(int), cmp_int);
            for (int k = 0; k < nc; k++) nd_order_set(c, comp + cs[k], cs[k + 1] - cs[k]);
            free(comp);
            free(cs);
            return;
        }
        free(comp);
        free(cs);
    }
    if (n <= c->leaf) {
        memcpy(c->perm + c->np, S, sizeof(int) * n);
        c->np += n;
        return;
    }
    int* lv = (int*)malloc(sizeof(int) * n);
    int* ls = (int*)malloc(sizeof(int) * (n + 2));
    int nl = nd_levels(c, S[0], sid, lv, ls);
    const int u = lv[ls[nl - 1]];
    nl = nd_levels(c, u, sid, lv, ls);
    const int h = nl - 1;
    if (h < 2) {
        memcpy(c->perm + c->np, S, sizeof(int) * n);
        c->np += n;
        free(lv);
        free(ls);
        return;
    }
    int best = -1;
    long long bk[4] = {0, 0, 0, 0};
    int A = 0;
    for (int m = 1; m < h; m++) {
        A += ls[m] - ls[m - 1];
        const int Lm = ls[m + 1] - ls[m], B = n - A - Lm;
        const int mn = A < B ? A : B;
        const int ok = 5LL * mn >= n;
        const int ab = A > B ? A - B : B - A;
        const long long key[4] = {ok ? 0 : 1, ok ? Lm : ab, ab, m};
        int less = best < 0;
        for (int q = 0; q < 4 && !less; q++) {
            if (key[q] < bk[q]) less = 1;
            if (key[q] != bk[q]) break;
        }
        if (less) {
            best = m;
            memcpy(bk, key, sizeof(bk));
        }
    }
    const int na = ls[best], nb = n - ls[best + 1], ns = ls[best + 1] - ls[best];
    int* Aset = (int*)malloc(sizeof(int) * (na + 1));
    int* Bset = (int*)malloc(sizeof(int) * (nb + 1));
    int* sep = (int*)malloc(sizeof(int) * (ns + 1));
    memcpy(Aset, lv, sizeof(int) * na);
    memcpy(sep, lv + ls[best], sizeof(int) * ns);
    memcpy(Bset, lv + ls[best + 1], sizeof(int) * nb);
    free(lv);
    free(ls);
    qsort(Aset, na, sizeof(int), cmp_int);
    qsort(Bset, nb, sizeof(int), cmp_int);
    nd_order_set(c, Aset, na);
    nd_order_set(c, Bset, nb);
    memcpy(c->perm + c->np, sep, sizeof(int) * ns);   /* L_m is sorted */
    c->np += ns;
    free(Aset);
    free(Bset);
    free(sep);
}

void ora_nd_order(int n, const int* adjStart, const int* adj, int leaf, int* perm)
{
    if (n <= 0 || !adjStart || !adj || !perm) return;
    nd_ctx c;
    c.as = adjStart;
    c.adj = adj;
    c.leaf = leaf;
    c.inS = (int*)calloc(n, sizeof(int));
    c.mark = (int*)calloc(n, sizeof(int));
    c.stamp = 0;
    c.perm = perm;
    c.np = 0;
    int* all = (int*)malloc(sizeof(int) * n);
    for (int i = 0; i < n; i++) all[i] = i;
    nd_order_set(&c, all, n);
    free(all);
    free(c.inS);
    free(c.mark);
}

/* ---- block-sparse LDL^T in a group order ---------------------------------------------- */
struct ora_sp {
    int n, g, ng;
    int* pos;      /* group -> elimination position */
    int* grp;      /* position -> group */
    int* rs;       /* position -> first permuted row; rs[ng] = n */
    int* cs;       /* row of positions P: cols[cs[P] .. cs[P+1]) sorted, cols[cs[P]] = P */
    int* cols;
    size_t* bo;    /* block offset (doubles) of entry e of cols */
    double* v;
};

static int sz_of(const ora_sp* s, int P) { return s->rs[P + 1] - s->rs[P]; }

static int find_col(const ora_sp* s, int P, int Q)
{
    int lo = s->cs[P], hi = s->cs[P + 1] - 1;
    while (lo <= hi) {
        const int m = (lo + hi) >> 1;
        if (s->cols[m] == Q) return m;
        if (s->cols[m] < Q) lo = m + 1;
        else hi = m - 1;
    }
    return -1;
}

ora_sp* ora_sp_create(int n, int g, const int* adjStart, const int* adj, const int* perm)
{
    ora_sp* s = (ora_sp*)calloc(1, sizeof(ora_sp));
    s->n = n;
    s->g = g;
    s->ng = (n + g - 1) / g;
    const int ng = s->ng;
    s->pos = (int*)malloc(sizeof(int) * (ng + 1));
    s->grp = (int*)malloc(sizeof(int) * (ng + 1));
    s->rs = (int*)malloc(sizeof(int) * (ng + 1));
    for (int P = 0; P < ng; P++) {
        s->grp[P] = perm[P];
        s->pos[perm[P]] = P;
    }
    s->rs[0] = 0;
    for (int P = 0; P < ng; P++) {
        const int q = s->grp[P];
        const int gs = n - q * g < g ? n - q * g : g;
        s->rs[P + 1] = s->rs[P] + gs;
    }
    /* symbolic: struct(P) = {P} u {adjacent Q > P}, then struct(parent) gains struct(P) \ {P, parent} */
    int** st = (int**)malloc(sizeof(int*) * ng);
    int* sn = (int*)calloc(ng, sizeof(int));
    int* sc = (int*)calloc(ng, sizeof(int));
    for (int P = 0; P < ng; P++) {
        const int q = s->grp[P];
        sc[P] = 8 + (adjStart[q + 1] - adjStart[q]);
        st[P] = (int*)malloc(sizeof(int) * sc[P]);
        st[P][sn[P]++] = P;
        for (int e = adjStart[q]; e < adjStart[q + 1]; e++) {
            const int Q = s->pos[adj[e]];
            if (Q > P) st[P][sn[P]++] = Q;
        }
    }
    for (int P = 0; P < ng; P++) {
        qsort(st[P], sn[P], sizeof(int), cmp_int);
        int m = 0;
        for (int t = 0; t < sn[P]; t++)
            if (m == 0 || st[P][t] != st[P][m - 1]) st[P][m++] = st[P][t];
        sn[P] = m;
        if (m > 1) {
            const int par = st[P][1];
            if (sn[par] + m > sc[par]) {
                sc[par] = 2 * (sn[par] + m);
                st[par] = (int*)realloc(st[par], sizeof(int) * sc[par]);
            }
            for (int t = 2; t < m; t++) st[par][sn[par]++] = st[P][t];
        }
    }
    s->cs = (int*)malloc(sizeof(int) * (ng + 1));
    size_t tot = 0;
    s->cs[0] = 0;
    for (int P = 0; P < ng; P++) s->cs[P + 1] = s->cs[P] + sn[P];
    s->cols = (int*)malloc(sizeof(int) * (s->cs[ng] + 1));
    s->bo = (size_t*)malloc(sizeof(size_t) * (s->cs[ng] + 1));
    for (int P = 0; P < ng; P++)
        for (int t = 0; t < sn[P]; t++) {
            const int e = s->cs[P] + t;
            s->cols[e] = st[P][t];
            s->bo[e] = tot;
            tot += (size_t)sz_of(s, P) * sz_of(s, st[P][t]);
        }
    s->v = (double*)calloc(tot + 1, sizeof(double));
    for (int P = 0; P < ng; P++) free(st[P]);
    free(st);
    free(sn);
    free(sc);
    return s;
}

void ora_sp_free(ora_sp* s)
{
    if (!s) return;
    free(s->pos); free(s->grp); free(s->rs); free(s->cs); free(s->cols); free(s->bo); free(s->v);
    free(s);
}

/* storage of system element (r, c), r <= c; the permutation may mirror it */
double* ora_sp_at(ora_sp* s, int r, int c)
{
    int P = s->pos[r / s->g], Q = s->pos[c / s->g], a = r % s->g, b = c % s->g;
    if (P > Q || (P == Q && a > b)) {
        int t = P; P = Q; Q = t;
        t = a; a = b; b = t;
    }
    const int e = find_col(s, P, Q);
    if (e < 0) return NULL;
    return &s->v[s->bo[e] + (size_t)a * sz_of(s, Q) + b];
}

int ora_sp_solve(ora_sp* s, const double* b, double* x)
{
    const int n = s->n, ng = s->ng;
    double* l = (double*)malloc(sizeof(double) * (n + 1));
    double* u = (double*)malloc(sizeof(double) * (n + 1));
    int* jcol = (int*)malloc(sizeof(int) * (n + 1));      /* permuted column of row k's entries */
    double** jp = (double**)malloc(sizeof(double*) * (n + 1));
    int* ent = (int*)malloc(sizeof(int) * (n + 1));        /* entry (block of row P) of each */
    int* tgt = NULL;
    size_t tcap = 0;
    int ok = 1;
    for (int P = 0; P < ng && ok; P++) {
        const int hP = sz_of(s, P), e0 = s->cs[P], e1 = s->cs[P + 1], ne = e1 - e0;
        /* target entries: block (cols[x], cols[y]), y >= x, in row cols[x] (merge walk) */
        if ((size_t)ne * ne > tcap) {
            tcap = (size_t)ne * ne;
            free(tgt);
            tgt = (int*)malloc(sizeof(int) * tcap);
        }
        for (int xq = 0; xq < ne; xq++) {
            const int R1 = s->cols[e0 + xq];
            int w = s->cs[R1];
            for (int yq = xq; yq < ne; yq++) {
                const int R2 = s->cols[e0 + yq];
                while (s->cols[w] < R2) w++;   /* the fill closure puts R2 in row R1 */
                tgt[(size_t)xq * ne + yq] = w;
            }
        }
        for (int a = 0; a < hP; a++) {
            const double d = s->v[s->bo[e0] + (size_t)a * hP + a];
            if (d == 0.0) {
                ok = 0;
                break;
            }
            /* row k's entries j > k, in ascending j: its diagonal block's right part, then the
             * blocks (P, Q > P) in ascending Q */
            int m = 0;
            for (int e = e0; e < e1; e++) {
                const int Q = s->cols[e], w = sz_of(s, Q);
                double* row = &s->v[s->bo[e] + (size_t)a * w];
                for (int bcol = (Q == P ? a + 1 : 0); bcol < w; bcol++) {
                    jcol[m] = s->rs[Q] + bcol;
                    jp[m] = &row[bcol];
                    ent[m] = e - e0;
                    u[m] = row[bcol];
                    l[m] = row[bcol] / d;
                    m++;
                }
            }
            for (int ii = 0; ii < m; ii++) {
                if (l[ii] == 0.0) continue;
                const int xq = ent[ii], R1 = s->cols[e0 + xq], ai = jcol[ii] - s->rs[R1];
                const double li = l[ii];
                /* targets (i, j), j >= i: entry by entry of row k */
                int jj = ii;
                while (jj < m) {
                    const int yq = ent[jj], R2 = s->cols[e0 + yq], w = sz_of(s, R2), c0 = s->rs[R2];
                    double* trow = &s->v[s->bo[tgt[(size_t)xq * ne + yq]] + (size_t)ai * w];
                    for (; jj < m && ent[jj] == yq; jj++) trow[jcol[jj] - c0] -= li * u[jj];
                }
            }
            for (int t = 0; t < m; t++) *jp[t] = l[t];   /* row k now holds L^T */
        }
    }
    free(tgt);
    free(u); free(jcol); free(jp); free(ent);
    if (!ok) {
        free(l);
        return 0;
    }
    /* L y = b (column sweep over row k's entries), y /= d, L^T x = y (row sweep, descending) */
    double* y = (double*)malloc(sizeof(double) * (n + 1));
    for (int P = 0; P < ng; P++) {
        const int q = s->grp[P];
        for (int a = 0; a < sz_of(s, P); a++) y[s->rs[P] + a] = b[q * s->g + a];
    }
    for (int P = 0; P < ng; P++) {
        const int hP = sz_of(s, P);
        for (int a = 0; a < hP; a++) {
            const int k = s->rs[P] + a;
            for (int e = s->cs[P]; e < s->cs[P + 1]; e++) {
                const int Q = s->cols[e], w = sz_of(s, Q);
                const double* row = &s->v[s->bo[e] + (size_t)a * w];
                for (int bcol = (Q == P ? a + 1 : 0); bcol < w; bcol++) y[s->rs[Q] + bcol] -= row[bcol] * y[k];
            }
        }
    }
    for (int P = 0; P < ng; P++)
        for (int a = 0; a < sz_of(s, P); a++)
            y[s->rs[P] + a] = y[s->rs[P] + a] / s->v[s->bo[s->cs[P]] + (size_t)a * sz_of(s, P) + a];
    for (int P = ng - 1; P >= 0; P--) {
        const int hP = sz_of(s, P);
        for (int a = hP - 1; a >= 0; a--) {
            const int i = s->rs[P] + a;
            double acc = y[i];
            for (int e = s->cs[P + 1] - 1; e >= s->cs[P]; e--) {
                const int Q = s->cols[e], w = sz_of(s, Q);
                const double* row = &s->v[s->bo[e] + (size_t)a * w];
                for (int bcol = w - 1; bcol >= (Q == P ? a + 1 : 0); bcol--) acc -= row[bcol] * y[s->rs[Q] + bcol];
            }
            y[i] = acc;
        }
    }
    for (int P = 0; P < ng; P++) {
        const int q = s->grp[P];
        for (int a = 0; a < sz_of(s, P); a++) x[q * s->g + a] = y[s->rs[P] + a];
    }
    free(y); free(l);
    return 1;
}

/* Dense-input unit form (tests): groups of 6 rows, adjacent when their block of the upper
 * triangle is nonzero; nested-dissection order (leaf 32); solve.  Returns 0 on a zero pivot. */
int ora_ldlt_solve_nd(const double* S, int n, const double* b, double* x)
{
    if (n <= 0) return 1;
    const int g = 6, ng = (n + g - 1) / g;
    int* deg = (int*)calloc(ng + 1, sizeof(int));
    unsigned char* nz = (unsigned char*)calloc((size_t)ng * ng, 1);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++)
            if (S[(size_t)i * n + j] != 0.0 && i / g != j / g) nz[(size_t)(i / g) * ng + j / g] = 1;
    for (int p = 0; p < ng; p++)
        for (int q = p + 1; q < ng; q++)
            if (nz[(size_t)p * ng + q]) { deg[p]++; deg[q]++; }
    int* as = (int*)malloc(sizeof(int) * (ng + 1));
    as[0] = 0;
    for (int p = 0; p < ng; p++) as[p + 1] = as[p] + deg[p];
    int* adj = (int*)malloc(sizeof(int) * (as[ng] + 1));
    int* f = (int*)malloc(sizeof(int) * (ng + 1));
    memcpy(f, as, sizeof(int) * ng);
    for (int p = 0; p < ng; p++)       /* lists come out sorted: p ascending, q ascending */
        for (int q = 0; q < ng; q++)
            if (p != q && nz[(size_t)(p < q ? p : q) * ng + (p < q ? q : p)]) adj[f[p]++] = q;
    int* perm = (int*)malloc(sizeof(int) * ng);
    ora_nd_order(ng, as, adj, 32, perm);
    ora_sp* s = ora_sp_create(n, g, as, adj, perm);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            double* t = ora_sp_at(s, i, j);
            if (t) *t = S[(size_t)i * n + j];
        }
    const int ok = ora_sp_solve(s, b, x);
    ora_sp_free(s);
    free(perm); free(f); free(adj); free(as); free(nz); free(deg);
    return ok;
}
