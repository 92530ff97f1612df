/*
 * psfm_knobs.h — C-ABI of the library's kernel-selection knobs (gfx950).
 *
 * A knob picks between measured implementations of one op (A/B runs, tests of a non-default
 * form).  Every knob is read ONCE, from the environment variable PSFM_<NAME>, when the library is
 * loaded; afterwards only psfm_knob_set changes it.  No kernel launch reads the environment, so a
 * stray variable set later cannot change which kernels run, and bench.py records every knob whose
 * value differs from its default (psfm_knob_* below) in its JSON line.
 *
 * Knobs (0 = the default policy unless stated):
 *   K12_PRIO   K12 wave-priority mode (default 2; 0 = no s_setprio; 1 refused) psfm_photometric.hip
 *   K12_PARTS  XCD parts per image of K12's work dealing (0 = 8 / B)        psfm_photometric.hip
 *   P3D_FWD    pack3d forward: 0 policy, 1 matrix cores, 2 VALU              psfm_pack3d.hip
 *   P3D_DX     pack3d input gradient: 0 policy, 1 matrix cores, 2 VALU       psfm_pack3d.hip
 *   P3D_DW     pack3d weight gradient: 0 policy, 1 VALU (generic)            psfm_pack3d.hip
 *   GN_PATH    GroupNorm: 0 resident where it fits, 1 two-pass everywhere   psfm_netops.hip
 *   BN_PATH    BatchNorm: 0 resident up to BN_RES_MAXM rows, MIOpen above       psfm_netops.hip
 *   BN_RES_MAXM  the largest M = N*H*W the resident BatchNorm takes (<= 8192) psfm_netops.hip
 *   GN_RES_RPT   most row vectors per thread of the resident GroupNorm (default 4) psfm_netops.hip
 * The environment accepts the integer or the value's name (e.g. PSFM_P3D_FWD=mfma).  A value the
 * knob does not have is refused with a line on stderr and kept by psfm_knob_rejected, so a run that
 * meant to select a form cannot silently run the default (bench.py lists it in config.knobs).
 *
 * Conventions as include/psfm.h.
 */
#ifndef PSFM_KNOBS_H
#define PSFM_KNOBS_H

#ifdef __cplusplus
extern "C" {
#endif

/* number of knobs; name / default / current value of knob i (NULL / 0 for i out of range) */
int psfm_knob_count(void);
const char* psfm_knob_name(int i);
int psfm_knob_default(int i);
int psfm_knob_value(int i);
/* the PSFM_<NAME> string the loader refused for knob i (NULL: none was refused) */
const char* psfm_knob_rejected(int i);

/* set a knob by name: 0, or -1 for an unknown name / a value outside the knob's range */
int psfm_knob_set(const char* name, int value);

#ifdef __cplusplus
}
#endif
#endif /* PSFM_KNOBS_H */
