// sm_hmc.cpp -- HMC driver layer of libsm_hip.so (include/sm_hip.h):
// HMC::HMC_algorithm (src/hmc.cpp:181-213) over the device-resident
// trajectory of sm_md.cpp, the reference's statistics (src/statistics.cpp),
// and the gauge-field gather behind SaveConf (src/gauge_conf.cpp:378-423).
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "sm_ctx.h"
#include "sm_fields.h"

using namespace sm;
using namespace sm_host;

namespace {

// mean() of include/statistics.h:9-16: sequential sum, then divide.
double seq_mean(const std::vector<double> &x) {
    double prom = 0;
    for (double v : x) prom += v * 1.0;
    return prom / x.size();
}

}  // namespace

extern "C" {

double sm_jackknife_error(const double *dat, int n, int bin) {
    // samples_mean + Jackknife_error, src/statistics.cpp:4-34, as written:
    // dat_bin = n / bin (integer), leave-one-block-out means over the first
    // bin*dat_bin samples, each divided by (n - dat_bin).
    if (!dat || n <= 0 || bin <= 0) return 0.0;
    const std::vector<double> v(dat, dat + n);
    const int dat_bin = n / bin;
    std::vector<double> means(bin);
    for (int i = 0; i < bin; i++) {
        double prom = 0;
        for (int k = 0; k < bin; k++)
            for (int j = k * dat_bin; j < k * dat_bin + dat_bin; j++)
                if (k != i) prom += v[j];
        means[i] = prom / (n - dat_bin);
    }
    const double normal_mean = seq_mean(v);
    double error = 0;
    for (int m = 0; m < bin; m++) error += (means[m] - normal_mean) * (means[m] - normal_mean);
    return std::sqrt(error * (bin - 1) / bin);
}

int sm_gather_gauge(sm_ctx *c, double *U0, double *U1) {
    TRY(check_ready(c));
    if (c->shard == 0 && (!U0 || !U1)) return fail(SM_ERR_ARG, "null argument on shard 0");
    HIP_TRY(hipSetDevice(c->device));
    const long V = c->g.V;
    const int P = c->nshard, Nx = c->g.Nx, Wt = c->g.Wt, Nt = c->g.Ntg;
    if (P == 1) return download_plane_pair(c, c->U, U0, U1);
    if (c->hosted) return fail(SM_ERR_STATE, "sm_gather_gauge needs the RCCL transport");
    const size_t cnt = (size_t)4 * V;  // doubles per shard: two planes of V complex
    double2 *buf = nullptr;
    if (c->shard == 0) {
        HIP_TRY(hipMalloc(&buf, sizeof(double) * cnt * P));
        HIP_TRY(hipMemcpyAsync(buf, c->U, sizeof(double) * cnt, hipMemcpyDeviceToDevice, c->stream));
    }
    {
        const int rc = rccl_gather_to0(c, c->stream, (const double *)c->U, (double *)buf, cnt);
        if (rc != SM_OK) {
            (void)hipStreamSynchronize(c->stream);
            if (buf) (void)hipFree(buf);
            return rc;
        }
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->shard == 0) {
        std::vector<double> h(cnt * P);
        const hipError_t e = hipMemcpy(h.data(), buf, sizeof(double) * cnt * P, hipMemcpyDeviceToHost);
        (void)hipFree(buf);
        HIP_TRY(e);
        // shard r holds global t in [r*Wt, (r+1)*Wt): local n = x*Wt + t
        for (int r = 0; r < P; r++) {
            const double *b = h.data() + cnt * r;
            for (int x = 0; x < Nx; x++)
                for (int t = 0; t < Wt; t++) {
                    const long nl = (long)x * Wt + t, ng = (long)x * Nt + (long)r * Wt + t;
                    U0[2 * ng] = b[2 * nl];
                    U0[2 * ng + 1] = b[2 * nl + 1];
                    U1[2 * ng] = b[2 * V + 2 * nl];
                    U1[2 * ng + 1] = b[2 * V + 2 * nl + 1];
                }
        }
    }
    return SM_OK;
}

int sm_hmc_run(sm_ctx *c, const sm_hmc_params *p, int hot_start, uint64_t first_traj, int Ntherm, int Nmeas,
               int Nsteps, const char *save_prefix, sm_hmc_summary *out, double *sp_series, double *gs_series) {
    if (!c || !p || !out) return fail(SM_ERR_ARG, "null argument");
    if (Ntherm < 0 || Nmeas < 1 || Nsteps < 0) return fail(SM_ERR_ARG, "Ntherm=%d Nmeas=%d Nsteps=%d", Ntherm, Nmeas,
                                                            Nsteps);
    // GaugeConf::initialization: random U(1) links (uniform angle), drawn here
    // on the device from a key no trajectory uses
    if (hot_start) TRY(sm_fill_gauge_dev(c, sm_traj_seed(p->seed, ~0ull), -1.0));
    TRY(check_ready(c));
    const double Ntot = (double)c->g.Nx * c->g.Ntg;
    uint64_t traj = first_traj;
    long accepted = 0, ntraj = 0, cg_it = 0;
    int cg_fail = 0;
    sm_hmc_result r;
    auto update = [&]() -> int {
        TRY(sm_hmc_trajectory(c, p, traj++, &r));
        ntraj++;
        cg_it += r.cg_iterations;
        cg_fail += r.cg_failures;
        return SM_OK;
    };
    for (int i = 0; i < Ntherm; i++) TRY(update());  // thermalisation
    std::vector<double> sp(Nmeas), gs(Nmeas);
    std::vector<double> U0, U1;
    for (int i = 0; i < Nmeas; i++) {
        TRY(update());
        accepted += r.accepted;
        sp[i] = r.sp;               // MeasureSp_HMC of the configuration kept
        gs[i] = r.gauge_action;     // Compute_gaugeAction
        if (save_prefix) {
            if (c->shard == 0 && U0.empty()) {
                U0.resize((size_t)4 * c->g.Nx * c->g.Ntg);
                U1.resize(U0.size());
            }
            TRY(sm_gather_gauge(c, c->shard == 0 ? U0.data() : nullptr, c->shard == 0 ? U1.data() : nullptr));
            if (c->shard == 0) {
                const std::string name = std::string(save_prefix) + "_" + std::to_string(i) + ".ctxt";
                TRY(sm_conf_write(name.c_str(), c->g.Nx, c->g.Ntg, U0.data(), U1.data()));
            }
        }
        if (i != Nmeas - 1)
            for (int j = 0; j < Nsteps; j++) {  // decorrelation
                TRY(update());
                accepted += r.accepted;
            }
    }
    out->Ep = seq_mean(sp) / (Ntot * 1.0);
    out->dEp = sm_jackknife_error(sp.data(), Nmeas, 20) / (Ntot * 1.0);
    out->gS = seq_mean(gs) / (Ntot * 1.0);
    out->dgS = sm_jackknife_error(gs.data(), Nmeas, 20) / (Ntot * 1.0);
    out->accepted = accepted;
    out->acceptance = accepted / ((Nmeas + Nsteps * (Nmeas - 1)) * 1.0);
    out->trajectories = ntraj;
    out->cg_iterations = cg_it;
    out->cg_failures = cg_fail;
    TRY(sm_cg_link_bytes(c, &out->cg_link_bytes));  // the link form the last solve's passes read (recorded at launch)
    if (sp_series)
        for (int i = 0; i < Nmeas; i++) sp_series[i] = sp[i];
    if (gs_series)
        for (int i = 0; i < Nmeas; i++) gs_series[i] = gs[i];
    return SM_OK;
}

}  // extern "C"
