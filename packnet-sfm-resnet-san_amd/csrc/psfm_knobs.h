// psfm_knobs.h — library-internal view of the kernel-selection knobs (include/psfm_knobs.h).
// The table lives in psfm_knobs.hip; it is filled from the environment once, by a load-time
// constructor, so host launch code reads a plain int (psfm::knob) and never the environment.
#pragma once

namespace psfm {

enum Knob {
    KNOB_K12_PRIO = 0,  // K12 wave-priority mode
    KNOB_K12_PARTS,     // XCD parts per image (0 = 8 / B)
    KNOB_P3D_FWD,       // 0 policy, 1 matrix cores, 2 VALU
    KNOB_P3D_DX,        // 0 policy, 1 matrix cores, 2 VALU (3 = grouped staging, A/B builds only)
    KNOB_P3D_DW,        // 0 policy, 1 VALU
    KNOB_GN_PATH,       // 0 resident where it fits, 1 two-pass
    KNOB_BN_PATH,       // 0 resident up to BN_RES_MAXM rows (the only form left; 1 / 2 removed in round 6)
    KNOB_BN_RES_MAXM,   // largest M = N*H*W the resident BatchNorm takes (<= 8192)
    KNOB_GN_RES_RPT,    // most row vectors per thread of the resident GroupNorm (1, 2, 4, 8)
    KNOB_COUNT
};

int knob(Knob k);

}  // namespace psfm
