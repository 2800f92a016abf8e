// oracle/hector_ref_harness.cc -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/libhector_logodds_ref.so).
//
// Compiles the REFERENCE log-odds cell functions unmodified, where they lie under /root/reference:
// lesson4/include/lesson4/hector_mapping/map/GridMapLogOdds.h (includes only <cmath>, :32).  No
// reference source is copied into this repository.  The rest of the Hector core needs Eigen3 (absent
// from the image, lesson4/CMakeLists.txt:26), so this header is the only part of the Hector path that
// can be built here; it pins rows A9 (log-odds cell ops) and the probability half of A7.
//
// Exported (extern "C", plain floats):
//   hlr_prob_to_logodds      GridMapLogOddsFunctions::probToLogOdds        GridMapLogOdds.h:153-157
//   hlr_factors              setUpdateFreeFactor / setUpdateOccupiedFactor :142-150 (ctor defaults :98-102)
//   hlr_apply_ops            updateSetOccupied / updateSetFree / updateUnsetFree on one cell  :108-129
//   hlr_grid_probability     getGridProbability                            :136-140
//   hlr_grid_probability_n   the same over an array
//   hlr_scan_probability     exhaustive comparison of getGridProbability against a candidate function
//                            over a range of float bit patterns (used to pin the oracle's restatement)
#include <cstdint>
#include <cstring>

#include "lesson4/hector_mapping/map/GridMapLogOdds.h"

namespace {
// probToLogOdds is protected: expose it through a subclass (the header itself is untouched)
struct Fn : public GridMapLogOddsFunctions {
    float p2l(float p) { return probToLogOdds(p); }
    float lf() const { return logOddsFree; }
    float lo() const { return logOddsOccupied; }
};
}  // namespace

extern "C" {

float hlr_prob_to_logodds(float prob)
{
    Fn f;
    return f.p2l(prob);
}

// factors (free, occupied) after the ctor (free_factor < 0: ctor defaults) or the two setters
void hlr_factors(float free_factor, float occ_factor, float *lf_out, float *lo_out)
{
    Fn f;
    if (free_factor >= 0.0f) {
        f.setUpdateFreeFactor(free_factor);
        f.setUpdateOccupiedFactor(occ_factor);
    }
    *lf_out = f.lf();
    *lo_out = f.lo();
}

// ops: 0 updateSetFree, 1 updateUnsetFree, 2 updateSetOccupied, 3 resetGridCell.  Returns the cell's
// final log-odds; *upd_out its updateIndex (only resetGridCell touches it here).
float hlr_apply_ops(float l0, int upd0, const int *ops, int nops, float free_factor, float occ_factor, int *upd_out)
{
    Fn f;
    if (free_factor >= 0.0f) {
        f.setUpdateFreeFactor(free_factor);
        f.setUpdateOccupiedFactor(occ_factor);
    }
    LogOddsCell c;
    c.set(l0);
    c.updateIndex = upd0;
    for (int i = 0; i < nops; ++i) {
        switch (ops[i]) {
        case 0: f.updateSetFree(c); break;
        case 1: f.updateUnsetFree(c); break;
        case 2: f.updateSetOccupied(c); break;
        default: c.resetGridCell(); break;
        }
    }
    if (upd_out) *upd_out = c.updateIndex;
    return c.getValue();
}

float hlr_grid_probability(float l)
{
    Fn f;
    LogOddsCell c;
    c.set(l);
    return f.getGridProbability(c);
}

void hlr_grid_probability_n(const float *l, float *out, long long n)
{
    Fn f;
    LogOddsCell c;
    for (long long i = 0; i < n; ++i) {
        c.set(l[i]);
        out[i] = f.getGridProbability(c);
    }
}

// Compare getGridProbability with cand(x) for every float whose bit pattern is in [bits_lo, bits_hi]
// (inclusive, one sign).  Returns the number of results that differ bit for bit; *first_bad gets the
// first differing pattern (0xFFFFFFFF if none).
long long hlr_scan_probability(uint32_t bits_lo, uint32_t bits_hi, float (*cand)(float), uint32_t *first_bad)
{
    Fn f;
    LogOddsCell c;
    long long bad = 0;
    *first_bad = 0xFFFFFFFFu;
    for (uint64_t b = bits_lo; b <= bits_hi; ++b) {
        float x;
        const uint32_t u = (uint32_t)b;
        memcpy(&x, &u, 4);
        c.set(x);
        const float r = f.getGridProbability(c), q = cand(x);
        uint32_t ur, uq;
        memcpy(&ur, &r, 4);
        memcpy(&uq, &q, 4);
        if (ur != uq) {
            if (!bad) *first_bad = u;
            ++bad;
        }
    }
    return bad;
}

}  // extern "C"
