// psfm_knobs.hip — the kernel-selection knobs (include/psfm_knobs.h): one table, filled from
// PSFM_<NAME> once when the library is loaded, changed afterwards only through psfm_knob_set.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/psfm_knobs.h"
#include "psfm_knobs.h"

#ifndef PSFM_K12_PRIO_DEFAULT
// K12 wave priority: mode 2 (p-eval at priority 0, the rest at 2; profiles/r04/prio)
#define PSFM_K12_PRIO_DEFAULT 2
#endif

#ifndef PSFM_BN_RES_MAXM_DEFAULT
// resident BatchNorm up to M = 2048 rows (ResNet18 layer3 / layer4 at B = 4, 192x640): interleaved
// A/B of the kitti-resnet-san step on one box (profiles/r05/bn): 2048 1076-1082 img/s, 8192 (layer2
// too: its 7680 rows x 16-byte per-lane row loads on 16 CUs run 22 / 41 us a launch) 1031, MIOpen's
// BatchNorm everywhere 1045-1048
#define PSFM_BN_RES_MAXM_DEFAULT 2048
#endif

namespace {

struct KnobDef {
    const char* name;
    int def, lo, hi;
    const char* values;  // comma-separated names of the values lo.. (empty: integers only)
    int value;
    int skip;              // a value inside [lo, hi] that is not a form (-1: none)
    const char* rejected;  // the PSFM_<NAME> string the loader refused (NULL: none)
};

constexpr int P3D_DX_HI = 2, BN_PATH_HI = 0;   // BN_PATH 1 / 2 (ticket / three-pass BatchNorm) were removed in round 6 (git 61b4f88 has them)

KnobDef g_knobs[psfm::KNOB_COUNT] = {
    // K12_PRIO: 0 off, 2 the p-eval at priority 0 and the rest at 2; the round-4 mode 1 is gone
    {"K12_PRIO", PSFM_K12_PRIO_DEFAULT, 0, 2, "", PSFM_K12_PRIO_DEFAULT, 1, nullptr},
    {"K12_PARTS", 0, 0, 8, "auto", 0, -1, nullptr},
    {"P3D_FWD", 0, 0, 2, "auto,mfma,valu", 0, -1, nullptr},
    {"P3D_DX", 0, 0, P3D_DX_HI, "auto,mfma,cl", 0, -1, nullptr},
    {"P3D_DW", 0, 0, 1, "auto,generic", 0, -1, nullptr},
    {"GN_PATH", 0, 0, 1, "resident,twopass", 0, -1, nullptr},
    {"BN_PATH", 0, 0, BN_PATH_HI, "resident", 0, -1, nullptr},
    {"BN_RES_MAXM", PSFM_BN_RES_MAXM_DEFAULT, 0, 8192, "", PSFM_BN_RES_MAXM_DEFAULT, -1, nullptr},
    // resident GroupNorm up to 4 row vectors per thread: RPT 8 (PackNetSAN01's 24x80 layers) ran
    // 18 / 29 us a launch and lost the interleaved A/B (profiles/r05/gn: kitti-packnet-san 373.3 vs
    // 375.6-376.7 img/s, kitti-packnet 286.9 vs 287.3)
    {"GN_RES_RPT", 4, 1, 8, "", 4, -1, nullptr},
};

// environment variables of forms that were removed (A/B variants of earlier rounds): a run that
// still sets one is told that it has no effect
const char* const g_retired[] = {"PSFM_GN_PIPE", "PSFM_GN_BLOCKS", "PSFM_AUGMENT_VEC", "PSFM_AUGMENT_NTH"};

bool accepted(const KnobDef& k, int v) { return v >= k.lo && v <= k.hi && v != k.skip; }

// value of a knob's environment string: one of its names (position = value) or an integer
bool parse(const KnobDef& k, const char* s, int& out) {
    const size_t n = strlen(s);
    int idx = k.lo;
    for (const char* p = k.values; *p; ++idx) {
        const char* e = strchr(p, ',');
        const size_t len = e ? (size_t)(e - p) : strlen(p);
        if (len == n && strncmp(p, s, n) == 0) {
            out = idx;
            return true;
        }
        if (!e) break;
        p = e + 1;
    }
    char* end = nullptr;
    const long v = strtol(s, &end, 10);
    if (end == s || *end) return false;
    out = (int)v;
    return true;
}

__attribute__((constructor)) void load_knobs() {
    for (KnobDef& k : g_knobs) {
        char var[64] = "PSFM_";
        strncat(var, k.name, sizeof(var) - 6);
        const char* s = getenv(var);
        if (!s) continue;
        int v;
        if (parse(k, s, v) && accepted(k, v)) {
            k.value = v;
        } else {
            k.rejected = s;
            fprintf(stderr, "psfm: ignoring %s=%s (not a value of this knob; it keeps %d)\n", var, s, k.value);
        }
    }
    for (const char* r : g_retired)
        if (getenv(r)) fprintf(stderr, "psfm: %s is set but that form was removed; it has no effect\n", r);
}

}  // namespace

namespace psfm {
int knob(Knob k) { return g_knobs[k].value; }
}  // namespace psfm

extern "C" {

int psfm_knob_count(void) { return psfm::KNOB_COUNT; }
const char* psfm_knob_name(int i) { return i >= 0 && i < psfm::KNOB_COUNT ? g_knobs[i].name : nullptr; }
int psfm_knob_default(int i) { return i >= 0 && i < psfm::KNOB_COUNT ? g_knobs[i].def : 0; }
int psfm_knob_value(int i) { return i >= 0 && i < psfm::KNOB_COUNT ? g_knobs[i].value : 0; }
const char* psfm_knob_rejected(int i) { return i >= 0 && i < psfm::KNOB_COUNT ? g_knobs[i].rejected : nullptr; }

int psfm_knob_set(const char* name, int value) {
    if (!name) return -1;
    for (KnobDef& k : g_knobs) {
        if (strcmp(k.name, name) == 0) {
            if (!accepted(k, value)) return -1;
            k.value = value;
            return 0;
        }
    }
    return -1;
}

}  // extern "C"
