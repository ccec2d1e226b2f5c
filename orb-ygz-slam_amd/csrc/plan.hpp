// plan.hpp — host-side extraction plan (see plan.cpp).
#pragma once
#include <stdio.h>

#include <vector>

#include "common.hpp"

namespace ygzfe {

struct ScaleInfo {
    float scale[kMaxLevels], inv_scale[kMaxLevels], sigma2[kMaxLevels], inv_sigma2[kMaxLevels];
    int budget[kMaxLevels];
    int umax[16];
};

struct PlanHost {
    Plan plan;
    ScaleInfo scales;
    std::vector<CellDesc> cells;
    std::vector<int> tabs;  // bilinear resize tables
};

void ic_umax(int umax[16]);  // IC_Angle circle rows (ORBextractor.cc:453-467)
void orb_scales(const ygzfe_orb_params &p, ScaleInfo *s);
int build_plan(const ygzfe_orb_params &p, int W, int H, PlanHost *ph, char *err, size_t errlen);

}  // namespace ygzfe
