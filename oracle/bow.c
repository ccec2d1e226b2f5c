/*
 * bow.c — CPU restatement of DBoW2's TemplatedVocabulary::transform as used by
 * Frame::ComputeBoW (Frame.cc:495-500: transform(desc, mBowVec, mFeatVec, 4)).
 * TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline); see ygz_oracle.h.
 *
 * Vocabulary structure as TemplatedVocabulary::loadFromTextFile builds it
 * (TemplatedVocabulary.h:1362-1448): node 0 is the root; node i >= 1 is
 * appended to children(parent[i]) in file order; a node flagged leaf gets the
 * next word id; Node() defaults word_id = 0, weight from the file.
 * isLeaf() = children.empty().
 *
 * transform(feature) (TemplatedVocabulary.h:1241-1281): from the root, descend
 * to the child with the smallest FORB::distance (FORB.cpp:82-101), first child
 * winning ties (`d < best_d`), until a node without children; nid = the node
 * reached at level L - levelsup.  transform(features, v, fv, levelsup)
 * (:1150-1212): features with weight > 0 are added — TF / TF_IDF:
 * v.addWeight (sum in feature order), IDF / BINARY: v.addIfNotExist; fv gets
 * (nid, feature index).  The scoring object decides normalisation
 * (ScoringObject.h:76-91: L1, L2, ChiSquare, KL, Bhattacharyya -> must,
 * L1 except L2; DotProduct -> none); without normalisation TF / TF_IDF
 * values are divided by v.size().  BowVector::normalize (BowVector.cpp:62-84):
 * L1 = sum of fabs in word order, L2 = sqrt(sum of squares); divide if > 0.
 */
#include "ygz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static int forb_distance(const uint8_t *a, const uint8_t *b) {
    int d = 0;
    for (int i = 0; i < 32; i += 4) {
        uint32_t x, y;
        memcpy(&x, a + i, 4);
        memcpy(&y, b + i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

struct ygzo_vocab {
    int k, L, scoring, weighting, n;
    int *child_ptr, *child, *word_id;
    uint8_t *desc;
    double *weight;
};

ygzo_vocab *ygzo_vocab_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t *parent,
                              const uint8_t *is_leaf, const uint8_t *desc, const double *weight) {
    if (n_nodes < 1) return NULL;
    ygzo_vocab *v = (ygzo_vocab *)calloc(1, sizeof(ygzo_vocab));
    v->k = k;
    v->L = L;
    v->scoring = scoring;
    v->weighting = weighting;
    v->n = n_nodes;
    v->child_ptr = (int *)calloc((size_t)n_nodes + 1, sizeof(int));
    v->child = (int *)calloc((size_t)n_nodes, sizeof(int));
    v->word_id = (int *)calloc((size_t)n_nodes, sizeof(int));
    v->desc = (uint8_t *)calloc((size_t)n_nodes, 32);
    v->weight = (double *)calloc((size_t)n_nodes, sizeof(double));
    for (int i = 1; i < n_nodes; i++) {
        if (parent[i] < 0 || parent[i] >= i) { ygzo_vocab_destroy(v); return NULL; }
        v->child_ptr[parent[i] + 1]++;
    }
    for (int i = 0; i < n_nodes; i++) v->child_ptr[i + 1] += v->child_ptr[i];
    int *fill = (int *)malloc(sizeof(int) * (size_t)n_nodes);
    memcpy(fill, v->child_ptr, sizeof(int) * (size_t)n_nodes);
    int words = 0;
    for (int i = 1; i < n_nodes; i++) {
        v->child[fill[parent[i]]++] = i;  /* children.push_back in node order */
        memcpy(v->desc + (size_t)i * 32, desc + (size_t)i * 32, 32);
        v->weight[i] = weight[i];
        if (is_leaf[i]) v->word_id[i] = words++;
    }
    free(fill);
    return v;
}

void ygzo_vocab_destroy(ygzo_vocab *v) {
    if (!v) return;
    free(v->child_ptr);
    free(v->child);
    free(v->word_id);
    free(v->desc);
    free(v->weight);
    free(v);
}

void ygzo_bow_transform_one(const ygzo_vocab *v, const uint8_t *f, int levelsup, int *word, double *weight,
                            int *nid) {
    const int nid_level = v->L - levelsup;
    if (nid_level <= 0) *nid = 0;
    int final_id = 0, level = 0;
    do {
        ++level;
        const int b = v->child_ptr[final_id], e = v->child_ptr[final_id + 1];
        final_id = v->child[b];
        double best_d = forb_distance(f, v->desc + (size_t)final_id * 32);
        for (int c = b + 1; c < e; c++) {
            const int id = v->child[c];
            const double d = forb_distance(f, v->desc + (size_t)id * 32);
            if (d < best_d) {
                best_d = d;
                final_id = id;
            }
        }
        if (level == nid_level) *nid = final_id;
    } while (v->child_ptr[final_id + 1] != v->child_ptr[final_id]);
    *word = v->word_id[final_id];
    *weight = v->weight[final_id];
}

static int cmp_int2(const void *a, const void *b) {
    const int *x = (const int *)a, *y = (const int *)b;
    if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
    return x[1] < y[1] ? -1 : (x[1] > y[1]);
}

int ygzo_compute_bow(const ygzo_vocab *v, const uint8_t *desc, int n, int levelsup, int32_t *bow_words,
                     double *bow_values, int *n_words, int32_t *fv_nodes, int32_t *fv_features, int *n_fv) {
    *n_words = 0;
    *n_fv = 0;
    if (n <= 0 || v->n <= 1) return 0;
    /* (word, feature) and (nid, feature) of the non-stopped features */
    int *wf = (int *)malloc(sizeof(int) * 2 * (size_t)n);
    double *ww = (double *)malloc(sizeof(double) * (size_t)n);
    int m = 0;
    for (int i = 0; i < n; i++) {
        int word = 0, nid = 0;
        double w = 0;
        ygzo_bow_transform_one(v, desc + (size_t)i * 32, levelsup, &word, &w, &nid);
        if (w > 0) {
            wf[2 * m] = word;
            wf[2 * m + 1] = i;
            ww[i] = w;
            fv_nodes[m] = nid;
            fv_features[m] = i;
            m++;
        }
    }
    /* FeatureVector: map<NodeId, vector<feature>> in (node, feature) order */
    int *nf = (int *)malloc(sizeof(int) * 2 * ((size_t)m + 1));
    for (int j = 0; j < m; j++) {
        nf[2 * j] = fv_nodes[j];
        nf[2 * j + 1] = fv_features[j];
    }
    qsort(nf, m, 2 * sizeof(int), cmp_int2);
    for (int j = 0; j < m; j++) {
        fv_nodes[j] = nf[2 * j];
        fv_features[j] = nf[2 * j + 1];
    }
    *n_fv = m;
    /* BowVector: map<WordId, WordValue>; a word's entries keep feature order */
    qsort(wf, m, 2 * sizeof(int), cmp_int2);
    const int tf = v->weighting == 0 /* TF_IDF */ || v->weighting == 1 /* TF */;
    int nw = 0;
    for (int j = 0; j < m; j++) {
        const double w = ww[wf[2 * j + 1]];
        if (nw > 0 && bow_words[nw - 1] == wf[2 * j]) {
            if (tf) bow_values[nw - 1] += w; /* addWeight; addIfNotExist keeps the first */
        } else {
            bow_words[nw] = wf[2 * j];
            bow_values[nw] = w;
            nw++;
        }
    }
    *n_words = nw;
    /* scoring: L1_NORM 0, L2_NORM 1, CHI_SQUARE 2, KL 3, BHATTACHARYYA 4, DOT_PRODUCT 5 */
    const int must = v->scoring != 5;
    const int l2 = v->scoring == 1;
    if (tf && nw > 0 && !must) {
        const double nd = nw;
        for (int j = 0; j < nw; j++) bow_values[j] /= nd;
    }
    if (must) {
        double norm = 0.0;
        if (!l2) {
            for (int j = 0; j < nw; j++) norm += fabs(bow_values[j]);
        } else {
            for (int j = 0; j < nw; j++) norm += bow_values[j] * bow_values[j];
            norm = sqrt(norm);
        }
        if (norm > 0.0)
            for (int j = 0; j < nw; j++) bow_values[j] /= norm;
    }
    free(wf);
    free(ww);
    free(nf);
    return nw;
}
