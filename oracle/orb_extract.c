/*
 * orb_extract.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * Restatement of ORB_SLAM2::ORBextractor (reference src/ORBextractor.cc,
 * include/ORBextractor.h).  Plain C, -ffp-contract=off.  Float/double
 * promotion follows the reference's C++ types expression by expression.
 */
#include "orb_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "brief_pattern.inc"

#define MAXL 32
#define PATCH_SIZE 31
#define HALF_PATCH_SIZE 15
#define EDGE_THRESHOLD 19

struct ora_extractor {
    int nfeatures, nlevels, iniThFAST, minThFAST;
    double scaleFactor;                  /* ORBextractor.h:105 (double member) */
    float scale[MAXL], invScale[MAXL], sigma2[MAXL], invSigma2[MAXL];
    int nPerLevel[MAXL];
    int umax[HALF_PATCH_SIZE + 1];
    /* pyramid: padded images (continuous, step = w+38), ORBextractor.cc:1107-1132 */
    uint8_t* padded[MAXL];
    int w[MAXL], h[MAXL];
    uint8_t* blurred[MAXL];              /* contiguous w x h (workingMat clone) */
    ora_kp* cand[MAXL];                  /* pre-octree candidates, absolute level coords */
    int ncand[MAXL], capcand[MAXL];
    int allocW, allocH;
};

/* ORBextractor ctor, ORBextractor.cc:410-470 */
ora_extractor* ora_extractor_new(int nfeatures, float scaleFactor, int nlevels,
                                 int iniThFAST, int minThFAST)
{
    if (nlevels < 1 || nlevels > MAXL) return NULL;
    ora_extractor* e = (ora_extractor*)calloc(1, sizeof(*e));
    e->nfeatures = nfeatures;
    e->scaleFactor = scaleFactor;
    e->nlevels = nlevels;
    e->iniThFAST = iniThFAST;
    e->minThFAST = minThFAST;
    e->scale[0] = 1.0f;
    e->sigma2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
        e->scale[i] = (float)(e->scale[i - 1] * e->scaleFactor);  /* float*double */
        e->sigma2[i] = e->scale[i] * e->scale[i];
    }
    for (int i = 0; i < nlevels; i++) {
        e->invScale[i] = 1.0f / e->scale[i];
        e->invSigma2[i] = 1.0f / e->sigma2[i];
    }
    float factor = (float)(1.0f / e->scaleFactor);
    float nDesired = nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        e->nPerLevel[l] = ora_cvRound_f(nDesired);
        sum += e->nPerLevel[l];
        nDesired *= factor;
    }
    e->nPerLevel[nlevels - 1] = nfeatures - sum > 0 ? nfeatures - sum : 0;

    /* umax, ORBextractor.cc:454-469 */
    int v, v0;
    int vmax = (int)floorf(HALF_PATCH_SIZE * sqrtf(2.f) / 2 + 1);
    int vmin = (int)ceilf(HALF_PATCH_SIZE * sqrtf(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    for (v = 0; v <= vmax; ++v) e->umax[v] = ora_cvRound_d(sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
        while (e->umax[v0] == e->umax[v0 + 1]) ++v0;
        e->umax[v] = v0;
        ++v0;
    }
    return e;
}

static void free_pyr(ora_extractor* e)
{
    for (int l = 0; l < MAXL; l++) {
        free(e->padded[l]); e->padded[l] = NULL;
        free(e->blurred[l]); e->blurred[l] = NULL;
        free(e->cand[l]); e->cand[l] = NULL;
        e->ncand[l] = e->capcand[l] = 0;
    }
}

void ora_extractor_free(ora_extractor* e)
{
    if (!e) return;
    free_pyr(e);
    free(e);
}

int ora_extractor_nlevels(const ora_extractor* e) { return e->nlevels; }

void ora_extractor_tables(const ora_extractor* e, float* scale, float* invScale,
                          float* sigma2, float* invSigma2, int* nPerLevel, int* umax16)
{
    for (int l = 0; l < e->nlevels; l++) {
        if (scale) scale[l] = e->scale[l];
        if (invScale) invScale[l] = e->invScale[l];
        if (sigma2) sigma2[l] = e->sigma2[l];
        if (invSigma2) invSigma2[l] = e->invSigma2[l];
        if (nPerLevel) nPerLevel[l] = e->nPerLevel[l];
    }
    if (umax16) memcpy(umax16, e->umax, sizeof(e->umax));
}

static inline int refl101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    }
    return p;
}

/* copyMakeBorder(.., EDGE_THRESHOLD x4, BORDER_REFLECT_101) into padded, interior already set */
static void make_border(uint8_t* pad, int w, int h)
{
    const int E = EDGE_THRESHOLD, pw = w + 2 * E;
    for (int y = 0; y < h + 2 * E; y++) {
        int sy = refl101(y - E, h);
        uint8_t* drow = pad + (size_t)y * pw;
        const uint8_t* srow = pad + (size_t)(sy + E) * pw + E;
        for (int x = 0; x < pw; x++) {
            if (y >= E && y < h + E && x >= E && x < w + E) continue;
            drow[x] = srow[refl101(x - E, w)];
        }
    }
}

/* ComputePyramid, ORBextractor.cc:1107-1132 */
static int compute_pyramid(ora_extractor* e, const uint8_t* img, int W, int H, int step)
{
    const int E = EDGE_THRESHOLD;
    for (int l = 0; l < e->nlevels; l++) {
        float sc = e->invScale[l];
        int w = ora_cvRound_f((float)W * sc), h = ora_cvRound_f((float)H * sc);
        if (w < 1 || h < 1) return -1;
        e->w[l] = w; e->h[l] = h;
        int pw = w + 2 * E, ph = h + 2 * E;
        free(e->padded[l]);
        e->padded[l] = (uint8_t*)malloc((size_t)pw * ph);
        uint8_t* interior = e->padded[l] + (size_t)E * pw + E;
        if (l == 0) {
            for (int y = 0; y < h; y++) memcpy(interior + (size_t)y * pw, img + (size_t)y * step, w);
        } else {
            const int ppw = e->w[l - 1] + 2 * E;
            const uint8_t* prev = e->padded[l - 1] + (size_t)E * ppw + E;
            ora_resize_linear_u8(prev, ppw, e->w[l - 1], e->h[l - 1], interior, pw, w, h);
        }
        make_border(e->padded[l], w, h);
    }
    return 0;
}

/* ------------------------------------------------------------------------
 * DistributeOctTree, ORBextractor.cc:539-763 (+ ExtractorNode::DivideNode 481-537)
 * std::list<ExtractorNode> is restated as an index-linked list.  The phase-2
 * sort key is (size, node pointer) in the reference; pointers order by heap
 * address, which is allocator-dependent.  We pin it to node creation order
 * (seq), the address order of a fresh heap -- see DESIGN.md Appendix quirks. */
typedef struct {
    int ULx, ULy, URx, URy, BLx, BLy, BRx, BRy;
    int* keys; int n;
    int noMore;
    long seq;
    int prev, next;
} onode;

typedef struct {
    onode* v; int n, cap;
    int head, size;
    long seq;
} olist;

static int olist_new_node(olist* L)
{
    if (L->n == L->cap) {
        L->cap = L->cap ? 2 * L->cap : 256;
        L->v = (onode*)realloc(L->v, sizeof(onode) * L->cap);
    }
    return L->n++;
}

static void olist_push_front(olist* L, int idx)
{
    onode* nd = &L->v[idx];
    nd->prev = -1;
    nd->next = L->head;
    if (L->head >= 0) L->v[L->head].prev = idx;
    L->head = idx;
    nd->seq = L->seq++;
    L->size++;
}

static void olist_push_back_init(olist* L, int idx, int* tail)
{
    onode* nd = &L->v[idx];
    nd->next = -1;
    nd->prev = *tail;
    if (*tail >= 0) L->v[*tail].next = idx; else L->head = idx;
    *tail = idx;
    nd->seq = L->seq++;
    L->size++;
}

static int olist_erase(olist* L, int idx)
{
    onode* nd = &L->v[idx];
    int nx = nd->next;
    if (nd->prev >= 0) L->v[nd->prev].next = nd->next; else L->head = nd->next;
    if (nd->next >= 0) L->v[nd->next].prev = nd->prev;
    free(nd->keys); nd->keys = NULL;
    L->size--;
    return nx;
}

/* DivideNode: children written as fresh pool nodes (not yet linked). */
static void divide_node(olist* L, int pidx, const ora_kp* K, int out[4])
{
    onode p = L->v[pidx];
    const int halfX = (int)ceilf((float)(p.URx - p.ULx) / 2);
    const int halfY = (int)ceilf((float)(p.BRy - p.ULy) / 2);
    int c[4];
    for (int i = 0; i < 4; i++) {
        c[i] = olist_new_node(L);
    }
    onode* n1 = &L->v[c[0]]; onode* n2 = &L->v[c[1]];
    onode* n3 = &L->v[c[2]]; onode* n4 = &L->v[c[3]];
    n1->ULx = p.ULx; n1->ULy = p.ULy;
    n1->URx = p.ULx + halfX; n1->URy = p.ULy;
    n1->BLx = p.ULx; n1->BLy = p.ULy + halfY;
    n1->BRx = p.ULx + halfX; n1->BRy = p.ULy + halfY;
    n2->ULx = n1->URx; n2->ULy = n1->URy;
    n2->URx = p.URx; n2->URy = p.URy;
    n2->BLx = n1->BRx; n2->BLy = n1->BRy;
    n2->BRx = p.URx; n2->BRy = p.ULy + halfY;
    n3->ULx = n1->BLx; n3->ULy = n1->BLy;
    n3->URx = n1->BRx; n3->URy = n1->BRy;
    n3->BLx = p.BLx; n3->BLy = p.BLy;
    n3->BRx = n1->BRx; n3->BRy = p.BLy;
    n4->ULx = n3->URx; n4->ULy = n3->URy;
    n4->URx = n2->BRx; n4->URy = n2->BRy;
    n4->BLx = n3->BRx; n4->BLy = n3->BRy;
    n4->BRx = p.BRx; n4->BRy = p.BRy;
    for (int i = 0; i < 4; i++) {
        onode* ch = &L->v[c[i]];
        ch->keys = (int*)malloc(sizeof(int) * (p.n > 0 ? p.n : 1));
        ch->n = 0; ch->noMore = 0; ch->prev = ch->next = -1;
    }
    const float n1URx = (float)L->v[c[0]].URx, n1BRy = (float)L->v[c[0]].BRy;
    for (int i = 0; i < p.n; i++) {
        const ora_kp* kp = &K[p.keys[i]];
        int dst;
        if (kp->x < n1URx) dst = (kp->y < n1BRy) ? 0 : 2;
        else dst = (kp->y < n1BRy) ? 1 : 3;
        onode* ch = &L->v[c[dst]];
        ch->keys[ch->n++] = p.keys[i];
    }
    for (int i = 0; i < 4; i++)
        if (L->v[c[i]].n == 1) L->v[c[i]].noMore = 1;
    for (int i = 0; i < 4; i++) out[i] = c[i];
}

typedef struct { int n; long seq; int idx; } size_ptr;
static int cmp_size_ptr(const void* a, const void* b)
{
    const size_ptr* x = (const size_ptr*)a; const size_ptr* y = (const size_ptr*)b;
    if (x->n != y->n) return x->n < y->n ? -1 : 1;
    if (x->seq != y->seq) return x->seq < y->seq ? -1 : 1;
    return 0;
}

/* Adds children with points to the list front (order n1..n4); records >1 ones. */
static void push_children(olist* L, const int ch[4], size_ptr** vs, int* nvs, int* capvs, int* nToExpand)
{
    for (int i = 0; i < 4; i++) {
        onode* c = &L->v[ch[i]];
        if (c->n > 0) {
            olist_push_front(L, ch[i]);
            if (c->n > 1) {
                if (nToExpand) (*nToExpand)++;
                if (*nvs == *capvs) { *capvs = *capvs ? 2 * *capvs : 64; *vs = (size_ptr*)realloc(*vs, sizeof(size_ptr) * *capvs); }
                (*vs)[*nvs].n = c->n; (*vs)[*nvs].seq = L->v[ch[i]].seq; (*vs)[*nvs].idx = ch[i];
                (*nvs)++;
            }
        } else {
            free(c->keys); c->keys = NULL;
        }
    }
}

static int distribute_octree(const ora_kp* K, int nK, int minX, int maxX, int minY, int maxY,
                             int N, ora_kp* out)
{
    const int nIni = (int)roundf((float)(maxX - minX) / (maxY - minY));
    if (nIni <= 0) return -1;  /* reference: UB (vpIniNodes of size 0), cannot occur at KITTI/EuRoC/TUM aspect */
    const float hX = (float)(maxX - minX) / nIni;
    olist L = {0};
    L.head = -1;
    int tail = -1;
    int* ini = (int*)malloc(sizeof(int) * nIni);
    for (int i = 0; i < nIni; i++) {
        int id = olist_new_node(&L);
        onode* nd = &L.v[id];
        nd->ULx = (int)(hX * (float)i); nd->ULy = 0;
        nd->URx = (int)(hX * (float)(i + 1)); nd->URy = 0;
        nd->BLx = nd->ULx; nd->BLy = maxY - minY;
        nd->BRx = nd->URx; nd->BRy = maxY - minY;
        nd->keys = (int*)malloc(sizeof(int) * (nK > 0 ? nK : 1));
        nd->n = 0; nd->noMore = 0;
        olist_push_back_init(&L, id, &tail);
        ini[i] = id;
    }
    for (int i = 0; i < nK; i++) {
        int b = (int)(size_t)(K[i].x / hX);
        onode* nd = &L.v[ini[b]];
        nd->keys[nd->n++] = i;
    }
    free(ini);
    int lit = L.head;
    while (lit >= 0) {
        onode* nd = &L.v[lit];
        if (nd->n == 1) { nd->noMore = 1; lit = nd->next; }
        else if (nd->n == 0) lit = olist_erase(&L, lit);
        else lit = nd->next;
    }

    int bFinish = 0;
    size_ptr* vs = NULL; int nvs = 0, capvs = 0;
    size_ptr* prev = NULL; int capprev = 0;
    while (!bFinish) {
        int prevSize = L.size;
        lit = L.head;
        int nToExpand = 0;
        nvs = 0;
        while (lit >= 0) {
            if (L.v[lit].noMore) { lit = L.v[lit].next; continue; }
            int ch[4];
            divide_node(&L, lit, K, ch);
            push_children(&L, ch, &vs, &nvs, &capvs, &nToExpand);
            lit = olist_erase(&L, lit);
        }
        if (L.size >= N || L.size == prevSize) {
            bFinish = 1;
        } else if ((L.size + nToExpand * 3) > N) {
            while (!bFinish) {
                prevSize = L.size;
                if (nvs > capprev) { capprev = nvs; prev = (size_ptr*)realloc(prev, sizeof(size_ptr) * capprev); }
                int nprev = nvs;
                memcpy(prev, vs, sizeof(size_ptr) * nvs);
                nvs = 0;
                qsort(prev, nprev, sizeof(size_ptr), cmp_size_ptr);
                for (int j = nprev - 1; j >= 0; j--) {
                    int ch[4];
                    divide_node(&L, prev[j].idx, K, ch);
                    push_children(&L, ch, &vs, &nvs, &capvs, NULL);
                    olist_erase(&L, prev[j].idx);
                    if (L.size >= N) break;
                }
                if (L.size >= N || L.size == prevSize) bFinish = 1;
            }
        }
    }

    int nout = 0;
    for (lit = L.head; lit >= 0; lit = L.v[lit].next) {
        onode* nd = &L.v[lit];
        int best = nd->keys[0];
        float maxResp = K[best].response;
        for (int k = 1; k < nd->n; k++)
            if (K[nd->keys[k]].response > maxResp) { best = nd->keys[k]; maxResp = K[best].response; }
        out[nout++] = K[best];
    }
    for (lit = L.head; lit >= 0; lit = L.v[lit].next) free(L.v[lit].keys);
    free(L.v); free(vs); free(prev);
    return nout;
}

/* IC_Angle, ORBextractor.cc:77-104 */
static float ic_angle(const uint8_t* img, int step, float px, float py, const int* umax)
{
    int m_01 = 0, m_10 = 0;
    const uint8_t* center = img + (size_t)ora_cvRound_f(py) * step + ora_cvRound_f(px);
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0;
        int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = center[u + v * step], val_minus = center[u - v * step];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return ora_fastAtan2((float)m_01, (float)m_10);
}

/* computeOrbDescriptor, ORBextractor.cc:108-147 */
static void orb_descriptor(const ora_kp* kp, const uint8_t* img, int step, uint8_t* desc)
{
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float angle = (float)kp->angle * factorPI;
    float a = ora_cosf(angle), b = ora_sinf(angle);
    const uint8_t* center = img + (size_t)ora_cvRound_f(kp->y) * step + ora_cvRound_f(kp->x);
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int k = 0; k < 8; k++) {
            int idx0 = i * 16 + 2 * k, idx1 = idx0 + 1;
            float x0 = (float)ORA_PATTERN_X[idx0], y0 = (float)ORA_PATTERN_Y[idx0];
            float x1 = (float)ORA_PATTERN_X[idx1], y1 = (float)ORA_PATTERN_Y[idx1];
            int t0 = center[ora_cvRound_f(x0 * b + y0 * a) * step + ora_cvRound_f(x0 * a - y0 * b)];
            int t1 = center[ora_cvRound_f(x1 * b + y1 * a) * step + ora_cvRound_f(x1 * a - y1 * b)];
            val |= (t0 < t1) << k;
        }
        desc[i] = (uint8_t)val;
    }
}

/* ComputeKeyPointsOctTree, ORBextractor.cc:765-853 (FAST part) */
static int cell_candidates(ora_extractor* e, int l)
{
    const int E = EDGE_THRESHOLD, pw = e->w[l] + 2 * E;
    const uint8_t* img = e->padded[l] + (size_t)E * pw + E;
    const float W = 30;
    const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
    const int maxBorderX = e->w[l] - EDGE_THRESHOLD + 3, maxBorderY = e->h[l] - EDGE_THRESHOLD + 3;
    const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
    const int nCols = (int)(width / W), nRows = (int)(height / W);
    if (nCols <= 0 || nRows <= 0) return -1;  /* reference divides by zero here */
    const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
    e->ncand[l] = 0;
    int cap = 4096;
    int* xs = (int*)malloc(sizeof(int) * cap * 3);
    int* ys = xs + cap; int* sc = ys + cap;
    for (int i = 0; i < nRows; i++) {
        const float iniY = (float)(minBorderY + i * hCell);
        float maxY = iniY + hCell + 6;
        if (iniY >= maxBorderY - 3) continue;
        if (maxY > maxBorderY) maxY = (float)maxBorderY;
        for (int j = 0; j < nCols; j++) {
            const float iniX = (float)(minBorderX + j * wCell);
            float maxX = iniX + wCell + 6;
            if (iniX >= maxBorderX - 6) continue;
            if (maxX > maxBorderX) maxX = (float)maxBorderX;
            const int r0 = (int)iniY, r1 = (int)maxY, c0 = (int)iniX, c1 = (int)maxX;
            const uint8_t* roi = img + (size_t)r0 * pw + c0;
            int n = ora_fast_roi(roi, pw, c1 - c0, r1 - r0, e->iniThFAST, xs, ys, sc, cap);
            if (n == 0) n = ora_fast_roi(roi, pw, c1 - c0, r1 - r0, e->minThFAST, xs, ys, sc, cap);
            if (n > cap) n = cap;
            for (int k = 0; k < n; k++) {
                if (e->ncand[l] == e->capcand[l]) {
                    e->capcand[l] = e->capcand[l] ? 2 * e->capcand[l] : 4096;
                    e->cand[l] = (ora_kp*)realloc(e->cand[l], sizeof(ora_kp) * e->capcand[l]);
                }
                ora_kp* kp = &e->cand[l][e->ncand[l]++];
                kp->x = (float)xs[k] + (float)(j * wCell);   /* ROI pt + cell offset (rel. minBorder) */
                kp->y = (float)ys[k] + (float)(i * hCell);
                kp->size = 7.f; kp->angle = -1; kp->response = (float)sc[k];
                kp->octave = 0; kp->class_id = -1;
            }
        }
    }
    free(xs);
    return 0;
}

/* operator(), ORBextractor.cc:1043-1105 */
int ora_extract(ora_extractor* e, const uint8_t* img, int W, int H, int step,
                ora_kp* kps, uint8_t* desc, int cap)
{
    if (!img || W <= 0 || H <= 0) return 0;
    if (compute_pyramid(e, img, W, H, step)) return -1;
    const int E = EDGE_THRESHOLD;
    ora_kp* lvl[MAXL];
    int nl[MAXL];
    int total = 0;
    for (int l = 0; l < e->nlevels; l++) {
        if (cell_candidates(e, l)) { for (int k = 0; k < l; k++) free(lvl[k]); return -1; }
        const int minBorderX = E - 3, minBorderY = minBorderX;
        const int maxBorderX = e->w[l] - E + 3, maxBorderY = e->h[l] - E + 3;
        lvl[l] = (ora_kp*)malloc(sizeof(ora_kp) * (e->ncand[l] + 1));
        nl[l] = distribute_octree(e->cand[l], e->ncand[l], minBorderX, maxBorderX, minBorderY,
                                  maxBorderY, e->nPerLevel[l], lvl[l]);
        if (nl[l] < 0) { for (int k = 0; k <= l; k++) free(lvl[k]); return -1; }
        const int scaledPatchSize = (int)(PATCH_SIZE * e->scale[l]);
        for (int i = 0; i < nl[l]; i++) {
            lvl[l][i].x += minBorderX;
            lvl[l][i].y += minBorderY;
            lvl[l][i].octave = l;
            lvl[l][i].size = (float)scaledPatchSize;
        }
        /* candidates kept in absolute level coords for stage tests */
        for (int i = 0; i < e->ncand[l]; i++) { e->cand[l][i].x += minBorderX; e->cand[l][i].y += minBorderY; }
        total += nl[l];
    }
    /* computeOrientation on the unblurred level */
    for (int l = 0; l < e->nlevels; l++) {
        const int pw = e->w[l] + 2 * E;
        const uint8_t* im = e->padded[l] + (size_t)E * pw + E;
        for (int i = 0; i < nl[l]; i++) lvl[l][i].angle = ic_angle(im, pw, lvl[l][i].x, lvl[l][i].y, e->umax);
    }
    if (total > cap) { for (int l = 0; l < e->nlevels; l++) free(lvl[l]); return -total; }
    int off = 0;
    for (int l = 0; l < e->nlevels; l++) {
        /* blurred clone is computed for every level (the reference skips empty levels;
         * output-equivalent) so stage tests can read it */
        const int pw = e->w[l] + 2 * E;
        free(e->blurred[l]);
        e->blurred[l] = (uint8_t*)malloc((size_t)e->w[l] * e->h[l]);
        ora_gaussian7_u8(e->padded[l] + (size_t)E * pw + E, pw, e->w[l], e->h[l], e->blurred[l], e->w[l]);
        for (int i = 0; i < nl[l]; i++)
            orb_descriptor(&lvl[l][i], e->blurred[l], e->w[l], desc + (size_t)(off + i) * 32);
        if (l != 0) {
            float s = e->scale[l];
            for (int i = 0; i < nl[l]; i++) { lvl[l][i].x *= s; lvl[l][i].y *= s; }
        }
        memcpy(kps + off, lvl[l], sizeof(ora_kp) * nl[l]);
        off += nl[l];
        free(lvl[l]);
    }
    return total;
}

int ora_extractor_level(const ora_extractor* e, int level, const uint8_t** data, int* pw, int* ph, int* step)
{
    if (level < 0 || level >= e->nlevels || !e->padded[level]) return -1;
    *data = e->padded[level];
    *pw = e->w[level] + 2 * EDGE_THRESHOLD;
    *ph = e->h[level] + 2 * EDGE_THRESHOLD;
    *step = *pw;
    return 0;
}

int ora_extractor_candidates(const ora_extractor* e, int level, ora_kp* out, int cap)
{
    if (level < 0 || level >= e->nlevels) return -1;
    int n = e->ncand[level];
    if (out) memcpy(out, e->cand[level], sizeof(ora_kp) * (n < cap ? n : cap));
    return n;
}

int ora_extractor_blurred(const ora_extractor* e, int level, const uint8_t** data, int* w, int* h)
{
    if (level < 0 || level >= e->nlevels || !e->blurred[level]) return -1;
    *data = e->blurred[level]; *w = e->w[level]; *h = e->h[level];
    return 0;
}
