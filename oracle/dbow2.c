/* dbow2.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's DBoW2 vocabulary
 * path (Thirdparty/DBoW2, vendored in the reference), the parity checker for the gfx950
 * ORBvocabulary kernels.  Never linked into the product library.
 *
 *   ora_voc_load_text      TemplatedVocabulary::loadFromTextFile   TemplatedVocabulary.h:1338-1424
 *                          FORB::fromString                         FORB.cpp:120-134
 *   ora_voc_transform_feature
 *                          transform(feature, word, weight, nid, levelsup)  TemplatedVocabulary.h:1217-1256
 *   ora_voc_transform      transform(features, BowVector, FeatureVector, levelsup) 1126-1197,
 *                          BowVector::addWeight/addIfNotExist/normalize BowVector.cpp:34-84,
 *                          FeatureVector::addFeature FeatureVector.cpp:31-45
 *   ora_voc_score_l1       L1Scoring::score                          ScoringObject.cpp:21-66
 *
 * Distances are FORB::distance (FORB.cpp:83-101), the 8-word popcount of a^b, compared as
 * double with a strict '<' so the first child of the smallest distance wins.
 *
 * The loader's trailing line.  saveToTextFile (1429-1449) ends every node line with endl, so
 * the loader's `while(!f.eof())` runs once more on an empty line: pid, nIsLeaf and the 32
 * descriptor tokens all fail to extract.  In the reference that is undefined behaviour (the
 * uninitialised locals keep whatever the previous iteration left in their stack slots; the
 * descriptor is an uninitialised cv::Mat).  Restated as the typical build realises it: the
 * extra node takes the previous line's parent and leaf flag, its descriptor bytes are zero
 * and its weight is 0 (Node()), so it is a stopped word.  Parity at this point is unpinned.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

typedef struct {
    int parent;
    int nchild, cap;
    int* child;
    uint8_t desc[32];
    double weight;
    int word_id;
} vnode;

struct ora_voc {
    int k, L, scoring, weighting;
    int nnodes, capn, nwords;
    vnode* nodes;
};

static int add_node(ora_voc* v) {
    if (v->nnodes == v->capn) {
        v->capn = v->capn ? 2 * v->capn : 1024;
        v->nodes = (vnode*)realloc(v->nodes, sizeof(vnode) * (size_t)v->capn);
    }
    vnode* n = &v->nodes[v->nnodes];
    memset(n, 0, sizeof(*n));
    return v->nnodes++;
}

static void add_child(vnode* p, int c) {
    if (p->nchild == p->cap) {
        p->cap = p->cap ? 2 * p->cap : 4;
        p->child = (int*)realloc(p->child, sizeof(int) * (size_t)p->cap);
    }
    p->child[p->nchild++] = c;
}

void ora_voc_free(ora_voc* v) {
    if (!v) return;
    for (int i = 0; i < v->nnodes; i++) free(v->nodes[i].child);
    free(v->nodes);
    free(v);
}

static int is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f'; }

/* next whitespace-separated token of *s (operator>> on a string), or NULL */
static const char* token(const char** s, int* len) {
    const char* p = *s;
    while (is_space(*p)) p++;
    if (!*p) { *s = p; return NULL; }
    const char* b = p;
    while (*p && !is_space(*p)) p++;
    *len = (int)(p - b);
    *s = p;
    return b;
}

static int tok_int(const char* t, int len, long* out) {
    char buf[64];
    if (len <= 0 || len >= 63) return 0;
    memcpy(buf, t, (size_t)len);
    buf[len] = 0;
    char* e;
    *out = strtol(buf, &e, 10);
    return e != buf;
}

ora_voc* ora_voc_load_text(const char* path, int* err) {
    *err = 0;
    FILE* f = fopen(path, "rb");
    if (!f) { *err = 1; return NULL; }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* buf = (char*)malloc((size_t)sz + 1);
    if (fread(buf, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); free(buf); *err = 1; return NULL; }
    fclose(f);
    buf[sz] = 0;
    ora_voc* v = (ora_voc*)calloc(1, sizeof(ora_voc));
    /* header: m_k m_L scoring weighting (1350-1364) */
    char* line = buf;
    char* nl = strchr(line, '\n');
    if (nl) *nl = 0;
    {
        const char* s = line;
        long x[4];
        for (int i = 0; i < 4; i++) {
            int len;
            const char* t = token(&s, &len);
            if (!t || !tok_int(t, len, &x[i])) { *err = 2; ora_voc_free(v); free(buf); return NULL; }
        }
        v->k = (int)x[0]; v->L = (int)x[1]; v->scoring = (int)x[2]; v->weighting = (int)x[3];
        if (v->k < 0 || v->k > 20 || v->L < 1 || v->L > 10 || v->scoring < 0 || v->scoring > 5 || v->weighting < 0 ||
            v->weighting > 3) {
            *err = 2; ora_voc_free(v); free(buf); return NULL;
        }
    }
    add_node(v);   /* root, id 0 */
    int prev_pid = 0, prev_leaf = 0;
    /* node lines, while(!f.eof()) (1375-1420): every line after the header, including the
     * empty one after a final '\n' */
    char* p = nl ? nl + 1 : NULL;
    while (p) {
        char* e = strchr(p, '\n');
        if (e) *e = 0;
        const char* s = p;
        int len;
        long pid = prev_pid, leaf = prev_leaf;
        const char* t = token(&s, &len);
        int ok = t && tok_int(t, len, &pid);
        if (ok) {
            t = token(&s, &len);
            ok = t && tok_int(t, len, &leaf);
        }
        if (!ok) { pid = prev_pid; leaf = prev_leaf; }   /* failed extraction: the UB realisation above */
        if (pid < 0 || pid >= v->nnodes) { *err = 3; ora_voc_free(v); free(buf); return NULL; }
        const int nid = add_node(v);
        vnode* n = &v->nodes[nid];
        n->parent = (int)pid;
        add_child(&v->nodes[pid], nid);
        if (ok) {
            for (int d = 0; d < 32; d++) {
                long x;
                t = token(&s, &len);
                if (t && tok_int(t, len, &x)) n->desc[d] = (uint8_t)x;   /* FORB::fromString: unset on failure */
            }
            t = token(&s, &len);
            if (t) {
                char wb[128];
                const int l2 = len < 127 ? len : 127;
                memcpy(wb, t, (size_t)l2);
                wb[l2] = 0;
                n->weight = strtod(wb, NULL);
            }
        }
        if (leaf > 0) n->word_id = v->nwords++;
        prev_pid = (int)pid;
        prev_leaf = (int)leaf;
        p = e ? e + 1 : NULL;
    }
    free(buf);
    return v;
}

void ora_voc_info(const ora_voc* v, int* k, int* L, int* scoring, int* weighting, int* nnodes, int* nwords) {
    *k = v->k; *L = v->L; *scoring = v->scoring; *weighting = v->weighting;
    *nnodes = v->nnodes; *nwords = v->nwords;
}

static int forb_distance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        uint32_t w = x ^ y;
        w = w - ((w >> 1) & 0x55555555u);
        w = (w & 0x33333333u) + ((w >> 2) & 0x33333333u);
        dist += (int)((((w + (w >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

/* transform(feature, word_id, weight, nid, levelsup), 1217-1256.  A leaf shallower than the
 * nid level leaves *nid unset in the reference (UB); restated as the leaf reached. */
void ora_voc_transform_feature(const ora_voc* v, const uint8_t* f, int levelsup, uint32_t* word, double* weight,
                               uint32_t* nid) {
    const int nid_level = v->L - levelsup;
    uint32_t nd = 0;
    int final_id = 0, level = 0;
    int set = nid_level <= 0;
    do {
        ++level;
        const vnode* n = &v->nodes[final_id];
        if (n->nchild == 0) break;   /* root without children: the callers return earlier */
        final_id = n->child[0];
        double best_d = (double)forb_distance(f, v->nodes[final_id].desc);
        for (int c = 1; c < n->nchild; c++) {
            const int id = n->child[c];
            const double d = (double)forb_distance(f, v->nodes[id].desc);
            if (d < best_d) { best_d = d; final_id = id; }
        }
        if (level == nid_level) { nd = (uint32_t)final_id; set = 1; }
    } while (v->nodes[final_id].nchild != 0);
    if (!set) nd = (uint32_t)final_id;
    *word = (uint32_t)v->nodes[final_id].word_id;
    *weight = v->nodes[final_id].weight;
    *nid = nd;
}

typedef struct {
    uint32_t key;
    int i;
    double w;
} kv;

static int cmp_kv(const void* a, const void* b) {
    const kv* x = (const kv*)a;
    const kv* y = (const kv*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->i < y->i ? -1 : (x->i > y->i);
}

/* transform(features, BowVector, FeatureVector, levelsup), 1126-1197.  BowVector as ascending
 * (word, value); FeatureVector as CSR (ascending node ids, features in insertion order,
 * fv_start has n_fv + 1 entries).  Returns 0, or -1 if the vocabulary is empty. */
int ora_voc_transform(const ora_voc* v, const uint8_t* desc, int N, int levelsup, uint32_t* bow_w, double* bow_v,
                      int* n_bow, uint32_t* fv_node, int* fv_start, int* fv_feat, int* n_fv) {
    *n_bow = 0;
    *n_fv = 0;
    fv_start[0] = 0;
    if (v->nwords == 0) return -1;
    const int must = v->scoring != 5;            /* every scoring but DOT_PRODUCT normalises */
    const int l2 = v->scoring == 1;              /* L2Scoring: L2 norm, the others L1 */
    kv* w = (kv*)malloc(sizeof(kv) * (size_t)(N > 0 ? N : 1));
    kv* nn = (kv*)malloc(sizeof(kv) * (size_t)(N > 0 ? N : 1));
    int m = 0;
    for (int i = 0; i < N; i++) {
        uint32_t word, nid;
        double wt;
        ora_voc_transform_feature(v, desc + 32 * (size_t)i, levelsup, &word, &wt, &nid);
        if (wt > 0) {
            w[m].key = word; w[m].i = i; w[m].w = wt;
            nn[m].key = nid; nn[m].i = i; nn[m].w = 0;
            m++;
        }
    }
    qsort(w, (size_t)m, sizeof(kv), cmp_kv);
    qsort(nn, (size_t)m, sizeof(kv), cmp_kv);
    const int tf = v->weighting == 0 || v->weighting == 1;   /* TF_IDF, TF: addWeight; else addIfNotExist */
    int nb = 0;
    for (int a = 0; a < m;) {
        int b;
        double s = w[a].w;
        for (b = a + 1; b < m && w[b].key == w[a].key; b++)
            if (tf) s += w[b].w;
        bow_w[nb] = w[a].key;
        bow_v[nb] = s;
        nb++;
        a = b;
    }
    if (tf && nb > 0 && !must) {
        const double nd = (double)nb;
        for (int a = 0; a < nb; a++) bow_v[a] /= nd;
    }
    if (must) {
        double norm = 0.0;
        if (!l2) {
            for (int a = 0; a < nb; a++) norm += fabs(bow_v[a]);
        } else {
            for (int a = 0; a < nb; a++) norm += bow_v[a] * bow_v[a];
            norm = sqrt(norm);
        }
        if (norm > 0.0)
            for (int a = 0; a < nb; a++) bow_v[a] /= norm;
    }
    int nf = 0;
    for (int a = 0; a < m;) {
        int b = a;
        fv_node[nf] = nn[a].key;
        fv_start[nf] = a;
        for (; b < m && nn[b].key == nn[a].key; b++) fv_feat[b] = nn[b].i;
        nf++;
        a = b;
    }
    fv_start[nf] = m;
    *n_bow = nb;
    *n_fv = nf;
    free(w);
    free(nn);
    return 0;
}

/* L1Scoring::score (ScoringObject.cpp:21-66) over two ascending BowVectors */
double ora_voc_score_l1(const uint32_t* w1, const double* v1, int n1, const uint32_t* w2, const double* v2, int n2) {
    double score = 0;
    int a = 0, b = 0;
    while (a < n1 && b < n2) {
        const double vi = v1[a], wi = v2[b];
        if (w1[a] == w2[b]) {
            score += fabs(vi - wi) - fabs(vi) - fabs(wi);
            ++a;
            ++b;
        } else if (w1[a] < w2[b]) {
            while (a < n1 && w1[a] < w2[b]) ++a;   /* v1.lower_bound(v2_it->first) */
        } else {
            while (b < n2 && w2[b] < w1[a]) ++b;
        }
    }
    score = -score / 2.0;
    return score;
}
