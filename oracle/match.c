/*
 * match.c — CPU restatement of the tracking-path ORBmatcher searches.
 * TEST INFRASTRUCTURE ONLY (parity oracle for csrc/match.hip); see ygz_oracle.h.
 *
 * Each search follows the reference loop literally: the frame grid of
 * Frame::AssignFeaturesToGrid / PosInGrid (Frame.cc:314-330, 483-493), the
 * candidate order of Frame::GetFeaturesInArea (Frame.cc:424-481: cells ix-major
 * then iy, indices in insertion order inside a cell), the strict-< best /
 * second-best updates, TH_HIGH / TH_LOW (ORBmatcher.cc:36-38), the nnratio
 * tests, the sequential "already matched" skips, the 30-bin rotation histogram
 * and ComputeThreeMaxima (:1471-1502).
 *
 * Inputs are what the reference reads from Frame / MapPoint, flattened: the
 * searched frame's keypoints, descriptors, mvuRight and image bounds; per
 * query the window (projection or vbPrevMatched), radius, level range, angle
 * and descriptor (MapPoint::GetDescriptor()), plus whether assigning it blocks
 * the keypoint for later queries (MapPoint::Observations() > 0).
 */
#include "ygz_oracle.h"

#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define GRID_COLS 64 /* FRAME_GRID_COLS (Frame.h:28) */
#define GRID_ROWS 48 /* FRAME_GRID_ROWS (Frame.h:27) */
#define TH_HIGH 100
#define TH_LOW 50
#define HISTO_LENGTH 30

typedef struct {
    float inv_w, inv_h;
    int start[GRID_COLS * GRID_ROWS + 1];
    int *idx;
} grid_t;

/* Frame.cc:296-297 */
static void grid_inv(const ygzo_mframe *f, float *iw, float *ih) {
    *iw = (float)GRID_COLS / (float)(f->max_x - f->min_x);
    *ih = (float)GRID_ROWS / (float)(f->max_y - f->min_y);
}

/* Frame::PosInGrid (Frame.cc:483-493): std::round(float) */
int ygzo_pos_in_grid(const ygzo_mframe *f, float x, float y, int *px, int *py) {
    float iw, ih;
    grid_inv(f, &iw, &ih);
    *px = (int)roundf((x - f->min_x) * iw);
    *py = (int)roundf((y - f->min_y) * ih);
    return !(*px < 0 || *px >= GRID_COLS || *py < 0 || *py >= GRID_ROWS);
}

/* Frame::AssignFeaturesToGrid (Frame.cc:314-330): cell (ix, iy) = slot ix*ROWS+iy */
static void grid_build(const ygzo_mframe *f, grid_t *g) {
    grid_inv(f, &g->inv_w, &g->inv_h);
    int *cell = (int *)malloc(sizeof(int) * (size_t)(f->n + 1));
    memset(g->start, 0, sizeof(g->start));
    for (int i = 0; i < f->n; i++) {
        int px, py;
        cell[i] = ygzo_pos_in_grid(f, f->kps[i].x, f->kps[i].y, &px, &py) ? px * GRID_ROWS + py : -1;
        if (cell[i] >= 0) g->start[cell[i] + 1]++;
    }
    for (int c = 0; c < GRID_COLS * GRID_ROWS; c++) g->start[c + 1] += g->start[c];
    int *fill = (int *)calloc(GRID_COLS * GRID_ROWS, sizeof(int));
    g->idx = (int *)malloc(sizeof(int) * (size_t)(f->n + 1));
    for (int i = 0; i < f->n; i++)
        if (cell[i] >= 0) g->idx[g->start[cell[i]] + fill[cell[i]]++] = i;
    free(fill);
    free(cell);
}

static void grid_free(grid_t *g) { free(g->idx); }

/* Frame::GetFeaturesInArea (Frame.cc:424-481); returns the count written to out */
static int features_in_area(const ygzo_mframe *f, const grid_t *g, float x, float y, float r, int minLevel,
                            int maxLevel, int *out) {
    int n = 0;
    const int nMinCellX = (int)floorf((x - f->min_x - r) * g->inv_w) > 0 ? (int)floorf((x - f->min_x - r) * g->inv_w) : 0;
    if (nMinCellX >= GRID_COLS) return 0;
    int nMaxCellX = (int)ceilf((x - f->min_x + r) * g->inv_w);
    if (nMaxCellX > GRID_COLS - 1) nMaxCellX = GRID_COLS - 1;
    if (nMaxCellX < 0) return 0;
    const int nMinCellY = (int)floorf((y - f->min_y - r) * g->inv_h) > 0 ? (int)floorf((y - f->min_y - r) * g->inv_h) : 0;
    if (nMinCellY >= GRID_ROWS) return 0;
    int nMaxCellY = (int)ceilf((y - f->min_y + r) * g->inv_h);
    if (nMaxCellY > GRID_ROWS - 1) nMaxCellY = GRID_ROWS - 1;
    if (nMaxCellY < 0) return 0;
    const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const int c = ix * GRID_ROWS + iy;
            for (int j = g->start[c]; j < g->start[c + 1]; j++) {
                const ygzo_kp *kp = &f->kps[g->idx[j]];
                if (bCheckLevels) {
                    if (kp->octave < minLevel) continue;
                    if (maxLevel >= 0 && kp->octave > maxLevel) continue;
                }
                const float distx = kp->x - x, disty = kp->y - y;
                if (fabsf(distx) < r && fabsf(disty) < r) out[n++] = g->idx[j];
            }
        }
    return n;
}

int ygzo_features_in_area(const ygzo_mframe *f, float x, float y, float r, int min_level, int max_level, int *out) {
    grid_t g;
    grid_build(f, &g);
    int n = features_in_area(f, &g, x, y, r, min_level, max_level, out);
    grid_free(&g);
    return n;
}

static inline int hamming(const uint8_t *a, const uint8_t *b) { return ygzo_descriptor_distance(a, b); }

/* ComputeThreeMaxima (ORBmatcher.cc:1471-1502) */
void ygzo_compute_three_maxima(const int *histo, int L, int *ind1, int *ind2, int *ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = histo[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            *ind3 = *ind2; *ind2 = *ind1; *ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            *ind3 = *ind2; *ind2 = i;
        } else if (s > max3) {
            max3 = s;
            *ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        *ind2 = -1;
        *ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        *ind3 = -1;
    }
}

/* the rotation bin (ORBmatcher.cc:1318-1323 and its copies): round(float) = roundf */
int ygzo_rot_bin(float angle_query, float angle_train) {
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = angle_query - angle_train;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

/* per-bin push lists of the rotation histogram (vector<int> rotHist[HISTO_LENGTH]) */
typedef struct { int *id, *bin, n; int count[HISTO_LENGTH + 34]; } rothist_t;

static void rot_init(rothist_t *h, int cap) {
    h->id = (int *)malloc(sizeof(int) * (size_t)(cap + 1));
    h->bin = (int *)malloc(sizeof(int) * (size_t)(cap + 1));
    h->n = 0;
    memset(h->count, 0, sizeof(h->count));
}
static void rot_push(rothist_t *h, int bin, int id) {
    h->id[h->n] = id;
    h->bin[h->n++] = bin;
    h->count[bin]++;
}
static void rot_free(rothist_t *h) { free(h->id); free(h->bin); }

/* SearchByProjection(CurrentFrame, LastFrame, th, bMono, checkLevel) (ORBmatcher.cc:1218-1350) and the
 * relocalisation form SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (:1352-1469):
 * best only, bestDist <= th_dist, rotation consistency.  train_match: -1 untouched, -2 set to NULL
 * by the rotation check, >= 0 the query assigned to CurrentFrame.mvpMapPoints[i2]. */
int ygzo_search_projection_best(const ygzo_mframe *cur, const ygzo_mquery *q, const uint8_t *q_desc, int nq,
                                const uint8_t *train_blocked, int th_dist, int check_ori, int32_t *train_match) {
    grid_t g;
    grid_build(cur, &g);
    uint8_t *blocked = (uint8_t *)calloc((size_t)cur->n + 1, 1);
    if (train_blocked) memcpy(blocked, train_blocked, (size_t)cur->n);
    for (int i = 0; i < cur->n; i++) train_match[i] = -1;
    int *cand = (int *)malloc(sizeof(int) * (size_t)(cur->n + 1));
    rothist_t rh;
    rot_init(&rh, nq);
    int nmatches = 0;
    for (int i = 0; i < nq; i++) {
        if (!(q[i].flags & YGZO_MQ_VALID)) continue;
        const int nc = features_in_area(cur, &g, q[i].u, q[i].v, q[i].radius, q[i].min_level, q[i].max_level, cand);
        if (nc == 0) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (int k = 0; k < nc; k++) {
            const int i2 = cand[k];
            if (blocked[i2]) continue;
            if ((q[i].flags & YGZO_MQ_STEREO) && cur->u_right && cur->u_right[i2] > 0) {
                const float er = fabsf(q[i].u_right - cur->u_right[i2]);
                if (er > q[i].radius) continue;
            }
            const int dist = hamming(q_desc + 32 * (size_t)i, cur->desc + 32 * (size_t)i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= th_dist) {
            train_match[bestIdx2] = i;
            blocked[bestIdx2] = (q[i].flags & YGZO_MQ_BLOCKS) ? 1 : 0;
            nmatches++;
            if (check_ori) rot_push(&rh, ygzo_rot_bin(q[i].angle, cur->kps[bestIdx2].angle), bestIdx2);
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        ygzo_compute_three_maxima(rh.count, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int p = 0; p < rh.n; p++)
                if (rh.bin[p] == b) {
                    train_match[rh.id[p]] = -2;
                    nmatches--;
                }
        }
    }
    rot_free(&rh);
    free(cand);
    free(blocked);
    grid_free(&g);
    return nmatches;
}

/* SearchByProjection(F, vpMapPoints, th, checkLevel) (ORBmatcher.cc:43-126): best and second best
 * with their octaves, bestDist <= TH_HIGH, nnratio test when both share a level. */
int ygzo_search_projection_ratio(const ygzo_mframe *F, const ygzo_mquery *q, const uint8_t *q_desc, int nq,
                                 const uint8_t *train_blocked, float nnratio, int32_t *train_match) {
    grid_t g;
    grid_build(F, &g);
    uint8_t *blocked = (uint8_t *)calloc((size_t)F->n + 1, 1);
    if (train_blocked) memcpy(blocked, train_blocked, (size_t)F->n);
    for (int i = 0; i < F->n; i++) train_match[i] = -1;
    int *cand = (int *)malloc(sizeof(int) * (size_t)(F->n + 1));
    int nmatches = 0;
    for (int i = 0; i < nq; i++) {
        if (!(q[i].flags & YGZO_MQ_VALID)) continue;
        const int nc = features_in_area(F, &g, q[i].u, q[i].v, q[i].radius, q[i].min_level, q[i].max_level, cand);
        if (nc == 0) continue;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int k = 0; k < nc; k++) {
            const int idx = cand[k];
            if (blocked[idx]) continue;
            if ((q[i].flags & YGZO_MQ_STEREO) && F->u_right && F->u_right[idx] > 0) {
                const float er = fabsf(q[i].u_right - F->u_right[idx]);
                if (er > q[i].radius) continue;
            }
            const int dist = hamming(q_desc + 32 * (size_t)i, F->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = F->kps[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = F->kps[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            train_match[bestIdx] = i;
            blocked[bestIdx] = (q[i].flags & YGZO_MQ_BLOCKS) ? 1 : 0;
            nmatches++;
        }
    }
    free(cand);
    free(blocked);
    grid_free(&g);
    return nmatches;
}

/* SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (ORBmatcher.cc:375-478).
 * prev_matched [2 n1] is updated in place (:472-475). */
int ygzo_search_for_initialization(const ygzo_mframe *F1, const ygzo_mframe *F2, float *prev_matched, int window,
                                   float nnratio, int check_ori, int32_t *matches12) {
    grid_t g;
    grid_build(F2, &g);
    int nmatches = 0;
    for (int i = 0; i < F1->n; i++) matches12[i] = -1;
    int *vMatchedDistance = (int *)malloc(sizeof(int) * (size_t)(F2->n + 1));
    int *vnMatches21 = (int *)malloc(sizeof(int) * (size_t)(F2->n + 1));
    for (int i = 0; i < F2->n; i++) { vMatchedDistance[i] = INT_MAX; vnMatches21[i] = -1; }
    int *cand = (int *)malloc(sizeof(int) * (size_t)(F2->n + 1));
    rothist_t rh;
    rot_init(&rh, F1->n);
    for (int i1 = 0; i1 < F1->n; i1++) {
        const int level1 = F1->kps[i1].octave;
        if (level1 > 0) continue;
        const int nc = features_in_area(F2, &g, prev_matched[2 * i1], prev_matched[2 * i1 + 1], (float)window, level1,
                                        level1, cand);
        if (nc == 0) continue;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int k = 0; k < nc; k++) {
            const int i2 = cand[k];
            const int dist = hamming(F1->desc + 32 * (size_t)i1, F2->desc + 32 * (size_t)i2);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) {
                    matches12[vnMatches21[bestIdx2]] = -1;
                    nmatches--;
                }
                matches12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (check_ori) rot_push(&rh, ygzo_rot_bin(F1->kps[i1].angle, F2->kps[bestIdx2].angle), i1);
            }
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        ygzo_compute_three_maxima(rh.count, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int p = 0; p < rh.n; p++)
                if (rh.bin[p] == b && matches12[rh.id[p]] >= 0) {
                    matches12[rh.id[p]] = -1;
                    nmatches--;
                }
        }
    }
    for (int i1 = 0; i1 < F1->n; i1++)
        if (matches12[i1] >= 0) {
            prev_matched[2 * i1] = F2->kps[matches12[i1]].x;
            prev_matched[2 * i1 + 1] = F2->kps[matches12[i1]].y;
        }
    rot_free(&rh);
    free(cand);
    free(vnMatches21);
    free(vMatchedDistance);
    grid_free(&g);
    return nmatches;
}

/* lower_bound over a node-sorted FeatureVector (std::map::lower_bound) */
static int fv_lower_bound(const int32_t *nodes, int n, int key) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) / 2;
        if (nodes[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* SearchByBoW(pKF, F, vpMapPointMatches) (ORBmatcher.cc:155-263).  FeatureVectors as node-sorted CSR:
 * node k = nodes[k], its features feats[ptr[k] .. ptr[k+1]).  f_match[F.N]: KF keypoint index or -1. */
int ygzo_search_by_bow(const ygzo_mframe *kf, const ygzo_mframe *F, const uint8_t *kf_usable, int n_kf_nodes,
                       const int32_t *kf_nodes, const int32_t *kf_ptr, const int32_t *kf_feats, int n_f_nodes,
                       const int32_t *f_nodes, const int32_t *f_ptr, const int32_t *f_feats, float nnratio,
                       int check_ori, int32_t *f_match) {
    for (int i = 0; i < F->n; i++) f_match[i] = -1;
    rothist_t rh;
    rot_init(&rh, F->n);
    int nmatches = 0;
    int KFit = 0, Fit = 0;
    while (KFit < n_kf_nodes && Fit < n_f_nodes) {
        if (kf_nodes[KFit] == f_nodes[Fit]) {
            for (int a = kf_ptr[KFit]; a < kf_ptr[KFit + 1]; a++) {
                const int realIdxKF = kf_feats[a];
                if (!kf_usable[realIdxKF]) continue; /* !pMP || pMP->isBad() */
                const uint8_t *dKF = kf->desc + 32 * (size_t)realIdxKF;
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                for (int b = f_ptr[Fit]; b < f_ptr[Fit + 1]; b++) {
                    const int realIdxF = f_feats[b];
                    if (f_match[realIdxF] >= 0) continue;
                    const int dist = hamming(dKF, F->desc + 32 * (size_t)realIdxF);
                    if (dist < bestDist1) {
                        bestDist2 = bestDist1;
                        bestDist1 = dist;
                        bestIdxF = realIdxF;
                    } else if (dist < bestDist2) {
                        bestDist2 = dist;
                    }
                }
                if (bestDist1 <= TH_LOW) {
                    if ((float)bestDist1 < nnratio * (float)bestDist2) {
                        f_match[bestIdxF] = realIdxKF;
                        if (check_ori)
                            rot_push(&rh, ygzo_rot_bin(kf->kps[realIdxKF].angle, F->kps[bestIdxF].angle), bestIdxF);
                        nmatches++;
                    }
                }
            }
            KFit++;
            Fit++;
        } else if (kf_nodes[KFit] < f_nodes[Fit]) {
            KFit += fv_lower_bound(kf_nodes + KFit, n_kf_nodes - KFit, f_nodes[Fit]);
        } else {
            Fit += fv_lower_bound(f_nodes + Fit, n_f_nodes - Fit, kf_nodes[KFit]);
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        ygzo_compute_three_maxima(rh.count, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int p = 0; p < rh.n; p++)
                if (rh.bin[p] == b) {
                    f_match[rh.id[p]] = -1;
                    nmatches--;
                }
        }
    }
    rot_free(&rh);
    return nmatches;
}
