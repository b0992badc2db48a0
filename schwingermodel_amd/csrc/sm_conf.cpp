// sm_conf.cpp -- the synthetic fields of the tests and the bench, and the
// reference's binary gauge-configuration format (src/gauge_conf.cpp
// SaveConf / readBinary): 28-byte records of x, t, mu (int32) and the link's
// real and imaginary parts (fp64), in x, t, mu order.

#include <cstdio>
#include <cstring>

#include "sm_ctx.h"
#include "sm_fields.h"

using namespace sm_host;

extern "C" {

void sm_fill_gauge(uint64_t seed, double sigma, int Nt_global, int x0, int nx, int t0, int Wt,
                   double *U0, double *U1) {
    sm_fields_fill_gauge(seed, sigma, Nt_global, x0, nx, t0, Wt, U0, U1);
}

void sm_fill_spinor(uint64_t seed, int Nt_global, int x0, int nx, int t0, int Wt, double *p0,
                    double *p1) {
    sm_fields_fill_spinor(seed, Nt_global, x0, nx, t0, Wt, p0, p1);
}

int sm_conf_write(const char *path, int Nx, int Nt, const double *U0, const double *U1) {
    FILE *f = fopen(path, "wb");
    if (!f) return fail(SM_ERR_ARG, "cannot open %s", path);
    unsigned char rec[28];
    for (int x = 0; x < Nx; x++)
        for (int t = 0; t < Nt; t++) {
            const long n = (long)x * Nt + t;
            for (int mu = 0; mu < 2; mu++) {
                const double *U = mu ? U1 : U0;
                memcpy(rec, &x, 4);
                memcpy(rec + 4, &t, 4);
                memcpy(rec + 8, &mu, 4);
                memcpy(rec + 12, &U[2 * n], 8);
                memcpy(rec + 20, &U[2 * n + 1], 8);
                if (fwrite(rec, 1, 28, f) != 28) {
                    fclose(f);
                    return fail(SM_ERR_ARG, "short write %s", path);
                }
            }
        }
    fclose(f);
    return SM_OK;
}

int sm_conf_read(const char *path, int Nx, int Nt, double *U0, double *U1) {
    FILE *f = fopen(path, "rb");
    if (!f) return fail(SM_ERR_ARG, "cannot open %s", path);
    unsigned char rec[28];
    // like readBinary (src/gauge_conf.cpp:515-531) the stored x/t/mu are not
    // trusted for placement: records are consumed in x, t, mu order.
    for (int x = 0; x < Nx; x++)
        for (int t = 0; t < Nt; t++) {
            const long n = (long)x * Nt + t;
            for (int mu = 0; mu < 2; mu++) {
                if (fread(rec, 1, 28, f) != 28) {
                    fclose(f);
                    return fail(SM_ERR_ARG, "%s: truncated at site %ld", path, n);
                }
                double *U = mu ? U1 : U0;
                memcpy(&U[2 * n], rec + 12, 8);
                memcpy(&U[2 * n + 1], rec + 20, 8);
            }
        }
    fclose(f);
    return SM_OK;
}

}  // extern "C"
