// Exhaustive check behind a candidate fast path of toPrecision(8)'s parse (js_number.h to_precision8,
// DESIGN.md §8): for every 8-digit integer n in [1e7, 1e8) and m in 0..22,
// and n = 1e8 (to_precision8_sl's carry keeps it), the quotient through the
// correctly rounded reciprocal R = RN(10^-m) and one fma correction of its remainder,
//     q0 = RN(n * R), q = RN(q0 + RN(n - q0 * 10^m) * R)   (the remainder term exact by fma),
// equals the IEEE quotient RN(n / 10^m).  Prints the mismatches per m (all 0).
#include <math.h>
#include <stdio.h>
#include <stdint.h>
int main(void) {
    static const double R[23] = {1e0, 1e-1, 1e-2, 1e-3, 1e-4, 1e-5, 1e-6, 1e-7, 1e-8, 1e-9, 1e-10, 1e-11, 1e-12,
                                 1e-13, 1e-14, 1e-15, 1e-16, 1e-17, 1e-18, 1e-19, 1e-20, 1e-21, 1e-22};
    static const double P[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12,
                                 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    long bad[23] = {0};
    #pragma omp parallel for schedule(dynamic)
    for (int m = 0; m <= 22; ++m) {
        long b = 0;
        for (int64_t n = 10000000; n <= 100000000; ++n) {
            const double x = (double)n;
            const double q0 = x * R[m];
            const double rem = fma(-q0, P[m], x);
            const double q = fma(rem, R[m], q0);
            if (q != x / P[m]) ++b;
        }
        bad[m] = b;
    }
    for (int m = 0; m <= 22; ++m) printf("m=%d bad=%ld\n", m, bad[m]);
    return 0;
}
