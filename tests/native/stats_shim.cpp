// CPU pinning shim (test infrastructure): exposes the product's host+device statistics header
// (csrc/fz_stats.h) to ctypes so tests/test_stats_pinning.py can compare it with scipy.
#include "fz_stats.h"

using namespace fz::stats;

extern "C" {
double shim_swilk(const double *y, long n, double *pw, int *ifault) { return swilk_sorted(y, n, pw, ifault); }
double shim_ppnd(double p) { return sw_ppnd(p); }
double shim_alnorm(double x, int upper) { return sw_alnorm(x, upper != 0); }
double shim_t_sf(double t, double df) { return t_sf(t, df); }
double shim_f1_sf(double w, double d) { return f1_sf(w, d); }
double shim_norm_sf(double z) { return norm_sf(z); }
double shim_log_ndtr(double a) { return log_ndtr(a); }
}
