/*
 * oracle/ldlt.c -- dense Bunch-Kaufman LDL^T (TEST INFRASTRUCTURE ONLY, see ora.h).
 *
 * Ipopt 3.12.8 factors its KKT matrix with MUMPS' symmetric indefinite LDL^T and
 * reads the inertia off D (Waechter & Biegler 2006, Sec. 3.1).  The oracle does
 * the same with a dense Bunch-Kaufman factorisation (partial pivoting with 1x1
 * and 2x2 pivots, alpha = (1+sqrt(17))/8), stored lower, 0-based, column-major.
 */
#include <math.h>
#include <string.h>
#include "ora.h"

#define A_(i, j) a[(size_t)(i) + (size_t)(j) * (size_t)n]

static int iamax_col(int n, const double* a, int j, int r0, int r1) {
    /* index of max |A(r,j)|, r in [r0, r1) */
    int best = r0;
    double bv = -1.0;
    for (int r = r0; r < r1; ++r) {
        double v = fabs(A_(r, j));
        if (v > bv) { bv = v; best = r; }
    }
    return best;
}

int ora_ldlt_factor(int n, double* a, int* ipiv, double tiny, int* npos, int* nneg, int* nzero) {
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    int pos = 0, neg = 0, zero = 0;
    int k = 0;
    while (k < n) {
        int kstep = 1, kp;
        double absakk = fabs(A_(k, k));
        int imax = k;
        double colmax = 0.0;
        if (k < n - 1) {
            imax = iamax_col(n, a, k, k + 1, n);
            colmax = fabs(A_(imax, k));
        }
        if (fmax(absakk, colmax) == 0.0) {
            kp = k;
        } else if (absakk >= alpha * colmax) {
            kp = k;
        } else {
            /* largest off-diagonal in row/column imax of the trailing matrix */
            double rowmax = 0.0;
            for (int j = k; j < imax; ++j) rowmax = fmax(rowmax, fabs(A_(imax, j)));
            for (int r = imax + 1; r < n; ++r) rowmax = fmax(rowmax, fabs(A_(r, imax)));
            if (absakk >= alpha * colmax * (colmax / rowmax)) {
                kp = k;
            } else if (fabs(A_(imax, imax)) >= alpha * rowmax) {
                kp = imax;
            } else {
                kp = imax;
                kstep = 2;
            }
        }
        int kk = k + kstep - 1;
        if (kp != kk) {
            /* symmetric interchange of rows/cols kk and kp inside A(k:n, k:n) */
            for (int r = kp + 1; r < n; ++r) {
                double t = A_(r, kk); A_(r, kk) = A_(r, kp); A_(r, kp) = t;
            }
            for (int j = kk + 1; j < kp; ++j) {
                double t = A_(j, kk); A_(j, kk) = A_(kp, j); A_(kp, j) = t;
            }
            double t = A_(kk, kk); A_(kk, kk) = A_(kp, kp); A_(kp, kp) = t;
            if (kstep == 2) {
                t = A_(k + 1, k); A_(k + 1, k) = A_(kp, k); A_(kp, k) = t;
            }
        }
        if (kstep == 1) {
            double d = A_(k, k);
            if (fabs(d) <= tiny) {
                ++zero;
                /* treat as exact zero: leave column unscaled (singular) */
                ipiv[k] = kp;
                k += 1;
                continue;
            }
            if (d > 0) ++pos; else ++neg;
            double d11 = 1.0 / d;
            for (int j = k + 1; j < n; ++j) {
                double xj = A_(j, k);
                if (xj != 0.0) {
                    double s = d11 * xj;
                    for (int r = j; r < n; ++r) A_(r, j) -= s * A_(r, k);
                }
            }
            for (int r = k + 1; r < n; ++r) A_(r, k) *= d11;
            ipiv[k] = kp;
        } else {
            double d11v = A_(k, k), d21v = A_(k + 1, k), d22v = A_(k + 1, k + 1);
            double det = d11v * d22v - d21v * d21v;
            if (fabs(det) <= tiny * tiny) {
                zero += 2;  /* degenerate 2x2 block */
            } else if (det < 0) {
                ++pos; ++neg;
            } else if (d11v + d22v > 0) {
                pos += 2;
            } else {
                neg += 2;
            }
            if (k < n - 2) {
                double D21 = A_(k + 1, k);
                double D11 = A_(k + 1, k + 1) / D21;
                double D22 = A_(k, k) / D21;
                double T = 1.0 / (D11 * D22 - 1.0);
                D21 = T / D21;
                for (int j = k + 2; j < n; ++j) {
                    double wk = D21 * (D11 * A_(j, k) - A_(j, k + 1));
                    double wkp1 = D21 * (D22 * A_(j, k + 1) - A_(j, k));
                    for (int r = j; r < n; ++r) A_(r, j) -= A_(r, k) * wk + A_(r, k + 1) * wkp1;
                    A_(j, k) = wk;
                    A_(j, k + 1) = wkp1;
                }
            }
            ipiv[k] = -(kp + 1);
            ipiv[k + 1] = -(kp + 1);
        }
        k += kstep;
    }
    *npos = pos;
    *nneg = neg;
    *nzero = zero;
    return zero == 0 ? 0 : 1;
}

void ora_ldlt_solve(int n, const double* a, const int* ipiv, double* b) {
    /* forward: L D y = P b */
    int k = 0;
    while (k < n) {
        if (ipiv[k] >= 0) {
            int kp = ipiv[k];
            if (kp != k) { double t = b[k]; b[k] = b[kp]; b[kp] = t; }
            double bk = b[k];
            for (int r = k + 1; r < n; ++r) b[r] -= A_(r, k) * bk;
            double d = A_(k, k);
            b[k] = (d != 0.0) ? bk / d : 0.0;
            k += 1;
        } else {
            int kp = -ipiv[k] - 1;
            if (kp != k + 1) { double t = b[k + 1]; b[k + 1] = b[kp]; b[kp] = t; }
            double b0 = b[k], b1 = b[k + 1];
            for (int r = k + 2; r < n; ++r) b[r] -= A_(r, k) * b0 + A_(r, k + 1) * b1;
            double akm1k = A_(k + 1, k);
            double akm1 = A_(k, k) / akm1k;
            double ak = A_(k + 1, k + 1) / akm1k;
            double denom = akm1 * ak - 1.0;
            double bkm1 = b0 / akm1k, bk = b1 / akm1k;
            b[k] = (ak * bkm1 - bk) / denom;
            b[k + 1] = (akm1 * bk - bkm1) / denom;
            k += 2;
        }
    }
    /* backward: L^T x = y, undo interchanges */
    k = n - 1;
    while (k >= 0) {
        if (ipiv[k] >= 0) {
            double s = 0.0;
            for (int r = k + 1; r < n; ++r) s += A_(r, k) * b[r];
            b[k] -= s;
            int kp = ipiv[k];
            if (kp != k) { double t = b[k]; b[k] = b[kp]; b[kp] = t; }
            k -= 1;
        } else {
            double s1 = 0.0, s0 = 0.0;
            for (int r = k + 1; r < n; ++r) {
                s1 += A_(r, k) * b[r];
                s0 += A_(r, k - 1) * b[r];
            }
            b[k] -= s1;
            b[k - 1] -= s0;
            int kp = -ipiv[k] - 1;
            if (kp != k) { double t = b[k]; b[k] = b[kp]; b[kp] = t; }
            k -= 2;
        }
    }
}

/* ---------------------------------------------------------------------------------
 * The same factorisation restricted to the matrix envelope: last[j] tracks the last
 * row of column j that can be nonzero (initialised from the matrix, widened by the
 * interchanges and by the fill of each elimination step), and every loop over rows
 * stops there.  The skipped operations subtract exact zeros, so for finite input the
 * pivots, the inertia and every stored value equal ora_ldlt_factor's bit for bit; for
 * a KKT matrix in stage order (a band of ~2.5 stages) the cost is O(n b^2) instead of
 * O(n^3).  Used by the structured CPU baseline (ora_ipm_opts.kkt_structured). */
int ora_ldlt_factor_env(int n, double* a, int* ipiv, double tiny, int* npos, int* nneg, int* nzero, int* last) {
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    int pos = 0, neg = 0, zero = 0;
    for (int j = 0; j < n; ++j) {
        int l = j;
        for (int r = n - 1; r > j; --r)
            if (A_(r, j) != 0.0) { l = r; break; }
        last[j] = l;
    }
    int k = 0;
    while (k < n) {
        int kstep = 1, kp;
        double absakk = fabs(A_(k, k));
        int imax = k;
        double colmax = 0.0;
        if (k < n - 1 && last[k] > k) {
            imax = iamax_col(n, a, k, k + 1, last[k] + 1);
            colmax = fabs(A_(imax, k));
        } else if (k < n - 1) {
            imax = k + 1;  /* (as iamax_col over an all-zero column) */
            colmax = 0.0;
        }
        if (fmax(absakk, colmax) == 0.0) {
            kp = k;
        } else if (absakk >= alpha * colmax) {
            kp = k;
        } else {
            double rowmax = 0.0;
            for (int j = k; j < imax; ++j)
                if (last[j] >= imax) rowmax = fmax(rowmax, fabs(A_(imax, j)));
            for (int r = imax + 1; r <= last[imax]; ++r) rowmax = fmax(rowmax, fabs(A_(r, imax)));
            if (absakk >= alpha * colmax * (colmax / rowmax)) {
                kp = k;
            } else if (fabs(A_(imax, imax)) >= alpha * rowmax) {
                kp = imax;
            } else {
                kp = imax;
                kstep = 2;
            }
        }
        int kk = k + kstep - 1;
        if (kp != kk) {
            const int lm = last[kk] > last[kp] ? last[kk] : last[kp];
            for (int r = kp + 1; r <= lm; ++r) {
                double t = A_(r, kk); A_(r, kk) = A_(r, kp); A_(r, kp) = t;
            }
            for (int j = kk + 1; j < kp; ++j) {
                double t = A_(j, kk); A_(j, kk) = A_(kp, j); A_(kp, j) = t;
                if (A_(kp, j) != 0.0 && last[j] < kp) last[j] = kp;
            }
            double t = A_(kk, kk); A_(kk, kk) = A_(kp, kp); A_(kp, kp) = t;
            if (kstep == 2) {
                t = A_(k + 1, k); A_(k + 1, k) = A_(kp, k); A_(kp, k) = t;
            }
            last[kk] = lm > kp ? lm : kp;
            last[kp] = lm;
            if (kstep == 2 && last[k] < kp) last[k] = kp;
        }
        if (kstep == 1) {
            double d = A_(k, k);
            if (fabs(d) <= tiny) {
                ++zero;
                ipiv[k] = kp;
                k += 1;
                continue;
            }
            if (d > 0) ++pos; else ++neg;
            double d11 = 1.0 / d;
            const int L = last[k];
            for (int j = k + 1; j <= L; ++j) {
                double xj = A_(j, k);
                if (xj != 0.0) {
                    double s = d11 * xj;
                    for (int r = j; r <= L; ++r) A_(r, j) -= s * A_(r, k);
                    if (last[j] < L) last[j] = L;
                }
            }
            for (int r = k + 1; r <= L; ++r) A_(r, k) *= d11;
            ipiv[k] = kp;
        } else {
            double d11v = A_(k, k), d21v = A_(k + 1, k), d22v = A_(k + 1, k + 1);
            double det = d11v * d22v - d21v * d21v;
            if (fabs(det) <= tiny * tiny) {
                zero += 2;
            } else if (det < 0) {
                ++pos; ++neg;
            } else if (d11v + d22v > 0) {
                pos += 2;
            } else {
                neg += 2;
            }
            const int L = last[k] > last[k + 1] ? last[k] : last[k + 1];
            if (k < n - 2) {
                double D21 = A_(k + 1, k);
                double D11 = A_(k + 1, k + 1) / D21;
                double D22 = A_(k, k) / D21;
                double T = 1.0 / (D11 * D22 - 1.0);
                D21 = T / D21;
                for (int j = k + 2; j <= L; ++j) {
                    double wk = D21 * (D11 * A_(j, k) - A_(j, k + 1));
                    double wkp1 = D21 * (D22 * A_(j, k + 1) - A_(j, k));
                    for (int r = j; r <= L; ++r) A_(r, j) -= A_(r, k) * wk + A_(r, k + 1) * wkp1;
                    A_(j, k) = wk;
                    A_(j, k + 1) = wkp1;
                    if (last[j] < L) last[j] = L;
                }
            }
            last[k] = last[k + 1] = L;
            ipiv[k] = -(kp + 1);
            ipiv[k + 1] = -(kp + 1);
        }
        k += kstep;
    }
    *npos = pos;
    *nneg = neg;
    *nzero = zero;
    return zero == 0 ? 0 : 1;
}

/* ora_ldlt_solve within the envelope of ora_ldlt_factor_env (same operations on the
 * nonzero entries, so the same result for finite data). */
void ora_ldlt_solve_env(int n, const double* a, const int* ipiv, const int* last, double* b) {
    int k = 0;
    while (k < n) {
        if (ipiv[k] >= 0) {
            int kp = ipiv[k];
            if (kp != k) { double t = b[k]; b[k] = b[kp]; b[kp] = t; }
            double bk = b[k];
            for (int r = k + 1; r <= last[k]; ++r) b[r] -= A_(r, k) * bk;
            double d = A_(k, k);
            b[k] = (d != 0.0) ? bk / d : 0.0;
            k += 1;
        } else {
            int kp = -ipiv[k] - 1;
            if (kp != k + 1) { double t = b[k + 1]; b[k + 1] = b[kp]; b[kp] = t; }
            double b0 = b[k], b1 = b[k + 1];
            for (int r = k + 2; r <= last[k]; ++r) b[r] -= A_(r, k) * b0 + A_(r, k + 1) * b1;
            double akm1k = A_(k + 1, k);
            double akm1 = A_(k, k) / akm1k;
            double ak = A_(k + 1, k + 1) / akm1k;
            double denom = akm1 * ak - 1.0;
            double bkm1 = b0 / akm1k, bk = b1 / akm1k;
            b[k] = (ak * bkm1 - bk) / denom;
            b[k + 1] = (akm1 * bk - bkm1) / denom;
            k += 2;
        }
    }
    k = n - 1;
    while (k >= 0) {
        if (ipiv[k] >= 0) {
            double s = 0.0;
            for (int r = k + 1; r <= last[k]; ++r) s += A_(r, k) * b[r];
            b[k] -= s;
            int kp = ipiv[k];
            if (kp != k) { double t = b[k]; b[k] = b[kp]; b[kp] = t; }
            k -= 1;
        } else {
            double s1 = 0.0, s0 = 0.0;
            for (int r = k + 1; r <= last[k]; ++r) {
                s1 += A_(r, k) * b[r];
                s0 += A_(r, k - 1) * b[r];
            }
            b[k] -= s1;
            b[k - 1] -= s0;
            int kp = -ipiv[k] - 1;
            if (kp != k) { double t = b[k]; b[k] = b[kp]; b[kp] = t; }
            k -= 2;
        }
    }
}
