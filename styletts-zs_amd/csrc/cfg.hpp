// Classifier-free guidance combine + Euler step of one sampler-state element, shared by
// stzs_cfg_euler (csrc/misc.hip): d = du + s (dc - du) with CFG, x' = x + dsig (x - d) / s0.
#pragma once
#include "common.hpp"

STZS_DEV float stzs_cfg_euler_elem(float xv, float dc, float du, int cfg, float s, float s0, float dsig) {
    const float d = cfg ? du + s * (dc - du) : dc;
    return xv + dsig * (xv - d) / s0;
}
