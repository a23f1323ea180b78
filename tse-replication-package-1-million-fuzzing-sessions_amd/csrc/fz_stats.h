// Special functions and test-statistic finishers, __host__ __device__ so the same code runs in the
// kernels and in the CPU pinning tests (tests/native/stats_shim.cpp compiles this header with g++).
//
// What each restates (third-party code the reference calls; scipy 1.15.3 / numpy 2.2.6 in this image):
//   swilk_*      scipy.stats.shapiro -> _ansari_swilk_statistics.swilk (Royston's AS R94 with
//                AS 111 `ppnd` and AS 66 `alnorm`); called at rq2_coverage_count.py:309,451.
//   t_sf         scipy.special.stdtr(df, -t): Student-t survival, via the regularised incomplete
//                beta I_x(df/2, 1/2) (spearmanr p at rq2_coverage_count.py:444, rq4b_coverage.py:888;
//                brunnermunzel p at rq3:349, rq4b:272,982).
//   f_sf         scipy.stats.f.sf(W, 1, d) (levene p, rq3:344, rq4b:275).
//   norm_sf      scipy.stats.norm.sf (mannwhitneyu asymptotic p, rq4b:265,268).
//   log_ndtr     scipy.special.log_ndtr (anderson, rq3:329,335).
#pragma once

#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define FZ_HD __host__ __device__
#else  // plain C++ (the CPU pinning shim)
#include <math.h>  // global isnan/isinf
#define FZ_HD
#endif

namespace fz {
namespace stats {

// ---------------------------------------------------------------------- Shapiro-Wilk (AS R94)
constexpr double kSwSmall = 1e-19;

// POLY(C, NORD, X) of AS R94: C[0] + x*(C[1] + x*(C[2] + ...)), evaluated from the top.
FZ_HD inline double sw_poly(const double *cc, int nord, double x) {
    double ret = cc[0];
    if (nord > 1) {
        double p = x * cc[nord - 1];
        for (int j = nord - 2; j > 0; --j) p = (p + cc[j]) * x;
        ret += p;
    }
    return ret;
}

// AS 111 (Beasley & Springer 1977): normal deviate for lower-tail probability p.
FZ_HD inline double sw_ppnd(double p) {
    const double split = 0.42;
    const double a0 = 2.50662823884, a1 = -18.61500062529, a2 = 41.39119773534, a3 = -25.44106049637;
    const double b1 = -8.47351093090, b2 = 23.08336743743, b3 = -21.06224101826, b4 = 3.13082909833;
    const double c0 = -2.78718931138, c1 = -2.29796479134, c2 = 4.85014127135, c3 = 2.32121276858;
    const double d1 = 3.54388924762, d2 = 1.63706781897;
    const double q = p - 0.5;
    if (fabs(q) <= split) {
        const double r = q * q;
        return q * (((a3 * r + a2) * r + a1) * r + a0) / ((((b4 * r + b3) * r + b2) * r + b1) * r + 1.0);
    }
    double r = p;
    if (q > 0.0) r = 1.0 - p;
    if (r <= 0.0) return 0.0;
    r = sqrt(-log(r));
    double v = (((c3 * r + c2) * r + c1) * r + c0) / ((d2 * r + d1) * r + 1.0);
    return q < 0.0 ? -v : v;
}

// AS 66 (Hill 1973): upper (or lower) tail of the standard normal.
FZ_HD inline double sw_alnorm(double x, bool upper) {
    const double ltone = 7.0, utzero = 18.66, con = 1.28;
    const double a1 = 5.75885480458, a2 = 2.62433121679, a3 = 5.92885724438;
    const double b1 = -29.8213557807, b2 = 48.6959930692;
    const double c1 = -3.8052e-8, c2 = 3.98064794e-4, c3 = -0.151679116635, c4 = 4.8385912808,
                 c5 = 0.742380924027, c6 = 3.99019417011;
    const double d1 = 1.00000615302, d2 = 1.98615381364, d3 = 5.29330324926, d4 = -15.1508972451,
                 d5 = 30.789933034;
    const double p = 0.398942280444, q = 0.39990348504, r = 0.398942280385;
    bool up = upper;
    double z = x;
    if (z < 0.0) {
        up = !up;
        z = -z;
    }
    double fn;
    if (z <= ltone || (up && z <= utzero)) {
        const double y = 0.5 * z * z;
        if (z > con)
            fn = r * exp(-y) / (z + c1 + d1 / (z + c2 + d2 / (z + c3 + d3 / (z + c4 + d4 / (z + c5 + d5 / (z + c6))))));
        else
            fn = 0.5 - z * (p - q * y / (y + a1 + b1 / (y + a2 + b2 / (y + a3))));
    } else {
        fn = 0.0;
    }
    return up ? fn : 1.0 - fn;
}

// m_i of AS R94 for 1-based i: ppnd((i - 0.375) / (n + 0.25)).
FZ_HD inline double sw_m(int64_t i, int64_t n) { return sw_ppnd((double(i) - 0.375) / (double(n) + 0.25)); }

// Per-sample coefficient scalars that depend only on n and summ2 = 2 * sum_{i<=n/2} m_i^2.
struct SwCoef {
    int64_t n;
    double a1, a2, fac;
    int i1;  // first 1-based index using -m_i / fac
};

FZ_HD inline SwCoef sw_coef(int64_t n, double summ2) {
    const double c1[6] = {0.0, 0.221157, -0.147981, -2.071190, 4.434685, -2.706056};
    const double c2[6] = {0.0, 0.042981, -0.293762, -1.752461, 5.682633, -3.582633};
    SwCoef c{n, 0.0, 0.0, 1.0, 2};
    if (n == 3) {
        c.a1 = 0.70710678118654752440;  // sqrt(1/2)
        c.i1 = 2;
        c.fac = 1.0;
        return c;
    }
    const double ssumm2 = sqrt(summ2);
    const double rsn = 1.0 / sqrt(double(n));
    const double m1 = sw_m(1, n);
    const double a1 = sw_poly(c1, 6, rsn) - m1 / ssumm2;
    c.a1 = a1;
    if (n > 5) {
        const double m2 = sw_m(2, n);
        const double a2 = -m2 / ssumm2 + sw_poly(c2, 6, rsn);
        c.a2 = a2;
        c.i1 = 3;
        c.fac = sqrt((summ2 - 2.0 * m1 * m1 - 2.0 * m2 * m2) / (1.0 - 2.0 * a1 * a1 - 2.0 * a2 * a2));
    } else {
        c.i1 = 2;
        c.fac = sqrt((summ2 - 2.0 * m1 * m1) / (1.0 - 2.0 * a1 * a1));
    }
    return c;
}

// A(k), 1-based k <= n/2.
FZ_HD inline double sw_a(const SwCoef &c, int64_t k) {
    if (k == 1) return c.a1;
    if (k == 2 && c.i1 == 3) return c.a2;
    if (c.n == 3) return 0.0;
    return -sw_m(k, c.n) / c.fac;
}

// sw_a from a precomputed normal score m = sw_m(k, n) (the same arithmetic, no ppnd call).
FZ_HD inline double sw_a_m(const SwCoef &c, int64_t k, double m) {
    if (k == 1) return c.a1;
    if (k == 2 && c.i1 == 3) return c.a2;
    if (c.n == 3) return 0.0;
    return -m / c.fac;
}

// Signed coefficient of the sample at sorted 1-based position i (mirror j = n + 1 - i).
FZ_HD inline double sw_coef_at(const SwCoef &c, int64_t i) {
    const int64_t j = c.n + 1 - i;
    if (i == j) return 0.0;
    const double a = sw_a(c, i < j ? i : j);
    return i > j ? a : -a;
}

// p-value of W (w1 = 1 - W as computed by the statistic loop).
FZ_HD inline double sw_pvalue(int64_t n, double w, double w1) {
    if (n == 3) {
        const double pi6 = 1.90985931710274, stqr = 1.04719755119660;
        double pw = pi6 * (asin(sqrt(w)) - stqr);
        return pw < 0.0 ? 0.0 : pw;
    }
    const double c3[4] = {0.5440, -0.39978, 0.025054, -6.714e-4};
    const double c4[4] = {1.3822, -0.77857, 0.062767, -0.0020322};
    const double c5[4] = {-1.5861, -0.31082, -0.083751, 0.0038915};
    const double c6[3] = {-0.4803, -0.082676, 0.0030302};
    const double g[2] = {-2.273, 0.459};
    const double an = double(n);
    double y = log(w1);
    const double xx = log(an);
    double m, s;
    if (n <= 11) {
        const double gamma = sw_poly(g, 2, an);
        if (y >= gamma) return kSwSmall;
        y = -log(gamma - y);
        m = sw_poly(c3, 4, an);
        s = exp(sw_poly(c4, 4, an));
    } else {
        m = sw_poly(c5, 4, xx);
        s = exp(sw_poly(c6, 3, xx));
    }
    // scipy's Cython port evaluates the upper normal tail to full double accuracy (it agrees with
    // ndtr(-z) to ~1e-11 on every case tried, where AS 66 alnorm is off by ~1e-8): use erfc.
    const double z = (y - m) / s;
    return 0.5 * erfc(z * 0.70710678118654752440);
}

// Sequential reference implementation over ascending y (already shifted by x[n/2] as scipy does).
// Returns W; *pw the p-value; *ifault 6 on zero range (then W = 1, p = 1 like scipy's init values).
FZ_HD inline double swilk_sorted(const double *y, int64_t n, double *pw, int *ifault) {
    *ifault = 0;
    double summ2 = 0.0;
    for (int64_t i = 1; i <= n / 2; ++i) {
        const double m = sw_m(i, n);
        summ2 += m * m;
    }
    summ2 *= 2.0;
    const SwCoef c = sw_coef(n, summ2);
    const double range = y[n - 1] - y[0];
    if (range < kSwSmall) {
        *ifault = 6;
        *pw = 1.0;
        return 1.0;
    }
    double sx = 0.0, sa = 0.0;
    for (int64_t i = 1; i <= n; ++i) {
        sx += y[i - 1] / range;
        sa += sw_coef_at(c, i);
    }
    sa /= double(n);
    sx /= double(n);
    double ssa = 0.0, ssx = 0.0, sax = 0.0;
    for (int64_t i = 1; i <= n; ++i) {
        const double asa = sw_coef_at(c, i) - sa;
        const double xsx = y[i - 1] / range - sx;
        ssa += asa * asa;
        ssx += xsx * xsx;
        sax += asa * xsx;
    }
    const double ssassx = sqrt(ssa * ssx);
    const double w1 = (ssassx - sax) * (ssassx + sax) / (ssa * ssx);
    const double w = 1.0 - w1;
    *pw = sw_pvalue(n, w, w1);
    return w;
}

// ------------------------------------------------------------------- incomplete beta & friends
// log(Gamma(a) / Gamma(a + b)) accurate for large a (Stirling difference) or via lgamma otherwise.
FZ_HD inline double lgamma_ratio(double a, double b) {
    if (a < 20.0) return lgamma(a) - lgamma(a + b);
    // (a-1/2)log a - (a+b-1/2)log(a+b) + b  + [series(a) - series(a+b)]
    const double ab = a + b;
    double r = -(a - 0.5) * log1p(b / a) - b * log(ab) + b;
    auto ser = [](double x) {
        const double x2 = 1.0 / (x * x);
        return (1.0 / 12.0 - x2 * (1.0 / 360.0 - x2 * (1.0 / 1260.0 - x2 * (1.0 / 1680.0)))) / x;
    };
    return r + ser(a) - ser(ab);
}

FZ_HD inline double lbeta(double a, double b) {
    // log B(a,b) = lgamma(b) + log(Gamma(a)/Gamma(a+b)), large argument first for accuracy
    if (a < b) {
        const double t = a;
        a = b;
        b = t;
    }
    return lgamma(b) + lgamma_ratio(a, b);
}

// a / b inside the continued fraction.  On the GPU a correctly rounded fp64 division is a chain of
// ~10 dependent instructions and the Lentz loop below is six of them per iteration on one thread
// (10-20 us per p-value at df ~ 1e3-1e6): there the reciprocal estimate, one Newton step and one
// residual correction of the quotient (within an ulp of a / b); on the host plain division.
FZ_HD inline double cf_div(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    const double q = a * r;
    return fma(fma(-b, q, a), r, q);
#else
    return a / b;
#endif
}

// Continued fraction of I_x(a,b) (modified Lentz), valid for x < (a+1)/(a+b+2).
FZ_HD inline double betacf(double a, double b, double x) {
    const double fpmin = 1e-300, eps = 3e-16;
    const double qab = a + b, qap = a + 1.0, qam = a - 1.0;
    double c = 1.0, d = 1.0 - qab * x / qap;
    if (fabs(d) < fpmin) d = fpmin;
    d = 1.0 / d;
    double h = d;
    for (int m = 1; m <= 100000; ++m) {
        const double m2 = 2.0 * m;
        double aa = cf_div(m * (b - m) * x, (qam + m2) * (a + m2));
        d = 1.0 + aa * d;
        if (fabs(d) < fpmin) d = fpmin;
        c = 1.0 + cf_div(aa, c);
        if (fabs(c) < fpmin) c = fpmin;
        d = cf_div(1.0, d);
        h *= d * c;
        aa = cf_div(-(a + m) * (qab + m) * x, (a + m2) * (qap + m2));
        d = 1.0 + aa * d;
        if (fabs(d) < fpmin) d = fpmin;
        c = 1.0 + cf_div(aa, c);
        if (fabs(c) < fpmin) c = fpmin;
        d = cf_div(1.0, d);
        const double del = d * c;
        h *= del;
        // (converged: the correction within an ulp of 1 - with the device's reciprocal-based
        // quotients the last factors may sit one ulp either side of 1 instead of on it)
        if (fabs(del - 1.0) < eps) break;
    }
    return h;
}

// Regularised incomplete beta I_x(a, b) with both x and y = 1 - x supplied (each computed
// directly by the caller, so neither loses accuracy near 0 or 1).
FZ_HD inline double ibeta_xy(double a, double b, double x, double y) {
    if (x <= 0.0) return 0.0;
    if (y <= 0.0) return 1.0;
    const double lx = y < 0.5 ? log1p(-y) : log(x);
    const double ly = x < 0.5 ? log1p(-x) : log(y);
    const double lbt = a * lx + b * ly - lbeta(a, b);
    if (x < (a + 1.0) / (a + b + 2.0)) return exp(lbt) * betacf(a, b, x) / a;
    return 1.0 - exp(lbt) * betacf(b, a, y) / b;  // symmetry: 1 - I_y(b, a)
}

// Student-t survival P(T > t), df > 0.  For t > 0: 0.5 * I_{df/(df+t^2)}(df/2, 1/2).
FZ_HD inline double t_sf(double t, double df) {
    if (isnan(t) || isnan(df) || !(df > 0.0)) return NAN;
    if (isinf(t)) return t > 0 ? 0.0 : 1.0;
    if (t == 0.0) return 0.5;
    const double at = fabs(t);
    const double t2 = at * at;
    double tail;
    if (isinf(t2)) {
        tail = 0.0;
    } else {
        const double x = df / (df + t2);
        const double y = t2 / (df + t2);
        tail = 0.5 * ibeta_xy(0.5 * df, 0.5, x, y);
    }
    return t > 0 ? tail : 1.0 - tail;
}

// F(1, d) survival at W >= 0:  I_{d/(d+W)}(d/2, 1/2)  (scipy fdtrc(1, d, W)).  Like cephes
// fdtrc, the argument is formed as w = d / (d + W) and 1 - w taken from that rounded w - when W
// is tiny against d this is what scipy returns (not the exact tail), and parity is with scipy.
FZ_HD inline double f1_sf(double W, double d) {
    if (isnan(W) || !(d > 0.0)) return NAN;
    if (W <= 0.0) return 1.0;
    if (isinf(W)) return 0.0;
    const double x = d / (d + W);
    return ibeta_xy(0.5 * d, 0.5, x, 1.0 - x);
}

FZ_HD inline double norm_sf(double z) { return 0.5 * erfc(z * 0.70710678118654752440); }

// log(Phi(a)).  scipy (xsf log_ndtr): log1p(-erfc(t)/2) for a >= -1, log(erfcx(-t)/2) - t^2
// below; here log(erfc(-t)/2) (same value) while erfc does not underflow, then the asymptotic
// series log(phi(a)/|a|) + log(1 - 1/a^2 + 3/a^4 - ...) for a <= -37.5.
FZ_HD inline double log_ndtr(double a) {
    const double t = a * 0.70710678118654752440;
    if (a >= -1.0) return log1p(-erfc(t) / 2.0);
    if (a > -37.5) return log(erfc(-t) / 2.0);
    const double x2 = 1.0 / (a * a);
    double term = 1.0, sum = 1.0;
    for (int k = 1; k < 12; ++k) {
        term *= -(2.0 * k - 1.0) * x2;
        sum += term;
    }
    return -0.5 * a * a - log(-a) - 0.91893853320467274178 + log(sum);
}

}  // namespace stats
}  // namespace fz
