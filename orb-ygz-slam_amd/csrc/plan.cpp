// plan.cpp — host-side planning of the extraction for one image size: level
// sizes, feature budgets, FAST cell grid, octree parameters, buffer slots.
// The float arithmetic restates ORBextractor.cc exactly (float products of
// the scale factor, cvRound = round-half-even), so the plan is identical to
// what the reference computes for the same parameters.
#include <math.h>
#include <float.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "plan.hpp"

namespace ygzfe {

static int cv_round_f(float v) { return (int)lrintf(v); }
static int cv_round_d(double v) { return (int)lrint(v); }

void orb_scales(const ygzfe_orb_params &p, ScaleInfo *s) {
    // ORBextractor.cc:416-445
    const double sf = (double)p.scale_factor;
    s->scale[0] = 1.0f;
    s->sigma2[0] = 1.0f;
    for (int i = 1; i < p.nlevels; i++) {
        s->scale[i] = (float)((double)s->scale[i - 1] * sf);
        s->sigma2[i] = s->scale[i] * s->scale[i];
    }
    for (int i = 0; i < p.nlevels; i++) {
        s->inv_scale[i] = 1.0f / s->scale[i];
        s->inv_sigma2[i] = 1.0f / s->sigma2[i];
    }
    const float factor = (float)(1.0 / sf);
    float desired = (float)p.nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)p.nlevels));
    int sum = 0;
    for (int l = 0; l < p.nlevels - 1; l++) {
        s->budget[l] = cv_round_f(desired);
        sum += s->budget[l];
        desired *= factor;
    }
    s->budget[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);
    ic_umax(s->umax);
}

// IC_Angle circle rows, ORBextractor.cc:453-467 (HALF_PATCH_SIZE = 15: the same for every config)
void ic_umax(int umax[16]) {
    const int vmax = (int)floorf(kHalfPatch * sqrtf(2.f) / 2 + 1);
    const int vmin = (int)ceilf(kHalfPatch * sqrtf(2.f) / 2);
    const double hp2 = kHalfPatch * kHalfPatch;
    int v, v0;
    for (v = 0; v <= vmax; ++v) umax[v] = cv_round_d(sqrt(hp2 - v * v));
    for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
}

// Path codes of k_octree_paths (extract.hip) as two tables per level: a key's code
// is X[x] | Y[y].  The x part carries the complemented root column on top; depth d's
// quadrant (bx | by << 1) goes at bits 30 - rb - 2d.., complemented at odd depths.
// The division midpoints follow ExtractorNode::DivideNode (ORBextractor.cc:481-482,
// ceil(half) of the integer extent) and the root columns DistributeOctTree
// (:537-559, hX in float, x / hX truncated).
static void octree_code_tables(LevelDesc &L, std::vector<int> *tabs) {
    const int nIni = L.n_ini, H0 = L.max_by - kMinBorder;
    const float hX = L.hX;
    const int rb = nIni > 1 ? 32 - __builtin_clz((unsigned)(nIni - 1)) : 0;
    const int ext = std::max((int)hX + 1, H0);
    const int Dn = std::min(32 - __builtin_clz((unsigned)ext) + 2, (32 - rb) >> 1);
    L.oct_rb = rb;
    L.oct_dn = Dn;
    L.oct_xtab = (int)tabs->size();
    for (int x = 0; x <= L.max_bx - kMinBorder; x++) {
        int idx = (int)((float)x / hX);
        idx = idx >= nIni ? nIni - 1 : idx;
        int x0 = (int)(hX * (float)idx), x1 = (int)(hX * (float)(idx + 1));
        uint32_t code = rb ? (uint32_t)(nIni - 1 - idx) << (32 - rb) : 0u;
        for (int d = 1, sh = 32 - rb - 2; d <= Dn; d++, sh -= 2) {
            const int mx = x0 + ((x1 - x0 + 1) >> 1);
            const bool bx = x >= mx;
            (bx ? x0 : x1) = mx;
            code |= (uint32_t)(bx ^ (d & 1)) << sh;
        }
        tabs->push_back((int)code);
    }
    L.oct_ytab = (int)tabs->size();
    for (int y = 0; y <= H0; y++) {
        int y0 = 0, y1 = H0;
        uint32_t code = 0u;
        for (int d = 1, sh = 32 - rb - 2; d <= Dn; d++, sh -= 2) {
            const int my = y0 + ((y1 - y0 + 1) >> 1);
            const bool by = y >= my;
            (by ? y0 : y1) = my;
            code |= (uint32_t)(by ^ (d & 1)) << (sh + 1);
        }
        tabs->push_back((int)code);
    }
}

int build_plan(const ygzfe_orb_params &p, int W, int H, PlanHost *ph, char *err, size_t errlen) {
    Plan &P = ph->plan;
    memset(&P, 0, sizeof(P));
    ph->cells.clear();
    ph->tabs.clear();
    if (p.nlevels < 1 || p.nlevels > kMaxLevels || p.nfeatures < 0 || !(p.scale_factor > 1.0f) || W < 8 ||
        H < 8) {
        snprintf(err, errlen, "invalid parameters (nlevels=%d nfeatures=%d scale=%g size=%dx%d)", p.nlevels,
                 p.nfeatures, (double)p.scale_factor, W, H);
        return -1;
    }
    ScaleInfo s;
    orb_scales(p, &s);
    ph->scales = s;
    P.W = W;
    P.H = H;
    P.nlevels = p.nlevels;
    P.ini_th = std::min(std::max(p.ini_th_fast, 0), 255);
    P.min_th = std::min(std::max(p.min_th_fast, 0), 255);
    P.blur_variant = p.blur_variant;
    for (int i = 0; i < 16; i++) P.umax[i] = s.umax[i];
    uint32_t off = 0;
    int cell_cap = 1, sel_total = 0, cand_total = 0, blur_tiles = 0, node_need = 0;
    for (int l = 0; l < p.nlevels; l++) {
        LevelDesc &L = P.lv[l];
        L.w = cv_round_f((float)W * s.inv_scale[l]);  // ORBextractor.cc:1131-1132
        L.h = cv_round_f((float)H * s.inv_scale[l]);
        if (L.w >= 4096 || L.h >= 4096 || L.w < 1 || L.h < 1) {
            snprintf(err, errlen, "level %d size %dx%d outside the supported 1..4095", l, L.w, L.h);
            return -1;
        }
        L.off = off;
        off += (uint32_t)L.w * (uint32_t)L.h;
        off = (off + 15u) & ~15u;  // 16-byte aligned level starts
        L.budget = s.budget[l];
        L.patch_size = (int)(kPatchSize * s.scale[l]);
        L.scale = s.scale[l];
        L.inv_scale = s.inv_scale[l];
        L.blur_tile_begin = blur_tiles;
        L.blur_tiles_x = (L.w + 255) / 256;  // k_blur7: one wave per 256 x kBlurRows strip
        L.blur_tiles_y = (L.h + kBlurRows - 1) / kBlurRows;
        blur_tiles += L.blur_tiles_x * L.blur_tiles_y;
        // resize mode (cv::resize, see oracle/orb.c ygzo_resize)
        if (l > 0) {
            const LevelDesc &S = P.lv[l - 1];
            const double inv_sx = (double)L.w / S.w, inv_sy = (double)L.h / S.h;
            const double sx = 1. / inv_sx, sy = 1. / inv_sy;
            const int isx = (int)lrint(sx), isy = (int)lrint(sy);
            const bool area_fast = fabs(sx - isx) < DBL_EPSILON && fabs(sy - isy) < DBL_EPSILON;
            if (area_fast && isx == 2 && isy == 2) {
                L.resize_mode = 1;
            } else {
                L.resize_mode = 2;
                L.xtab_off = (int)ph->tabs.size();
                L.xmax = L.w;
                for (int dx = 0; dx < L.w; dx++) {
                    float fx = (float)((dx + 0.5) * sx - 0.5);
                    int ix = (int)floorf(fx);
                    fx -= ix;
                    if (ix < 0) fx = 0, ix = 0;
                    if (ix + 1 >= S.w) {
                        if (dx < L.xmax) L.xmax = dx;
                        if (ix >= S.w - 1) fx = 0, ix = S.w - 1;
                    }
                    const int a0 = std::min(std::max(cv_round_f((1.f - fx) * 2048), -32768), 32767);
                    const int a1 = std::min(std::max(cv_round_f(fx * 2048), -32768), 32767);
                    ph->tabs.push_back(ix);
                    ph->tabs.push_back((int)(((uint32_t)(uint16_t)a0) | ((uint32_t)(uint16_t)a1 << 16)));
                }
                L.ytab_off = (int)ph->tabs.size();
                for (int dy = 0; dy < L.h; dy++) {
                    float fy = (float)((dy + 0.5) * sy - 0.5);
                    int iy = (int)floorf(fy);
                    fy -= iy;
                    const int b0 = std::min(std::max(cv_round_f((1.f - fy) * 2048), -32768), 32767);
                    const int b1 = std::min(std::max(cv_round_f(fy * 2048), -32768), 32767);
                    ph->tabs.push_back(std::min(std::max(iy, 0), S.h - 1));
                    ph->tabs.push_back(std::min(std::max(iy + 1, 0), S.h - 1));
                    ph->tabs.push_back((int)(((uint32_t)(uint16_t)b0) | ((uint32_t)(uint16_t)b1 << 16)));
                }
            }
        }
        // FAST cell grid (ORBextractor.cc:728-781)
        const float Wc = 30;
        const int minB = kMinBorder, maxBX = L.w - kEdgeThreshold + 3, maxBY = L.h - kEdgeThreshold + 3;
        L.max_bx = maxBX;
        L.max_by = maxBY;
        const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
        const int nCols = (int)(width / Wc), nRows = (int)(height / Wc);
        L.cell_begin = (int)ph->cells.size();
        if (nCols > 0 && nRows > 0) {
            const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
            for (int i = 0; i < nRows; i++) {
                const float iniY = (float)(minB + i * hCell);
                float maxY = iniY + hCell + 6;
                if (iniY >= maxBY - 3) continue;
                if (maxY > maxBY) maxY = (float)maxBY;
                for (int j = 0; j < nCols; j++) {
                    const float iniX = (float)(minB + j * wCell);
                    float maxX = iniX + wCell + 6;
                    if (iniX >= maxBX - 6) continue;
                    if (maxX > maxBX) maxX = (float)maxBX;
                    CellDesc c;
                    c.x0 = (int16_t)(int)iniX;
                    c.y0 = (int16_t)(int)iniY;
                    c.rw = (int16_t)((int)maxX - (int)iniX);
                    c.rh = (int16_t)((int)maxY - (int)iniY);
                    c.offx = (int16_t)(j * wCell);
                    c.offy = (int16_t)(i * hCell);
                    c.level = (int16_t)l;
                    c.pad = 0;
                    if (c.rw > kMaxRoi || c.rh > kMaxRoi) {
                        snprintf(err, errlen, "FAST cell ROI %dx%d exceeds %d", c.rw, c.rh, kMaxRoi);
                        return -1;
                    }
                    const int iw = std::max(c.rw - 6, 0), ih = std::max(c.rh - 6, 0);
                    cell_cap = std::max(cell_cap, ((iw + 1) / 2) * ((ih + 1) / 2));
                    P.fast_S = std::max(P.fast_S, ((std::max((int)c.rw, (int)c.rh) + 3) / 4) * 4);
                    L.fast_roi = std::max(L.fast_roi, std::max((int)c.rw, (int)c.rh));
                    L.fast_rw = std::max(L.fast_rw, (int)c.rw);
                    L.fast_rh = std::max(L.fast_rh, (int)c.rh);
                    ph->cells.push_back(c);
                }
            }
        }
        L.ncells = (int)ph->cells.size() - L.cell_begin;
        // DistributeOctTree initial nodes (ORBextractor.cc:537-539)
        int nIni = (int)roundf((float)(maxBX - minB) / (maxBY - minB));
        if (nIni < 1) nIni = 1;
        if (nIni > 8) {
            snprintf(err, errlen, "level %d aspect ratio needs %d initial octree nodes (max 8)", l, nIni);
            return -1;
        }
        L.n_ini = nIni;
        L.hX = (float)(maxBX - minB) / nIni;
        octree_code_tables(L, &ph->tabs);
        L.sel_cap = std::max(L.budget + 4, 4 * nIni + 4) + 8;
        L.sel_off = sel_total;
        sel_total += L.sel_cap;
        node_need = std::max(node_need, L.budget + 4 * nIni + 16);
    }
    // candidate slots need the per-cell capacity: second pass
    for (int l = 0; l < p.nlevels; l++) {
        LevelDesc &L = P.lv[l];
        L.cand_cap = std::max(L.ncells * cell_cap, 1);
        L.cand_off = cand_total;
        cand_total += L.cand_cap;
    }
    P.pyr_bytes = off + 64;  // tail padding: dword row gathers may read up to 11 bytes past a window
    P.fast_S = std::max(P.fast_S, 8);
    P.ncells = (int)ph->cells.size();
    P.cell_cap = cell_cap;
    P.sel_total = sel_total;
    P.cand_total = cand_total;
    P.kp_cap = sel_total;
    P.blur_tiles = blur_tiles;
    if (node_need <= 512) P.node_cap = 512;
    else if (node_need <= 1024) P.node_cap = 1024;
    else if (node_need <= 2048) P.node_cap = 2048;
    else {
        snprintf(err, errlen, "per-level feature budget too large for the octree node pool (need %d > 2048)",
                 node_need);
        return -1;
    }
    if (ph->tabs.empty()) ph->tabs.push_back(0);
    return 0;
}

}  // namespace ygzfe
