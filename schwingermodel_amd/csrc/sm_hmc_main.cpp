// sm_hmc_main.cpp -- `sm_hmc`: the reference's HMC program (src/main.cpp)
// on MI355X, one MPI rank per GPU, the whole HMC resident on the device
// through libsm_hip.so (sm_hmc_run: device trajectories, Dirac/CG kernels,
// RCCL halos over xGMI).
//
//   mpirun -n P ./sm_hmc <Nx> <Nt> [seed] [--even-odd]  < params
//
// stdin takes the reference's parameters in its order (src/main.cpp:30-53):
// ranks_x ranks_t m0 MD_steps trajectory_length beta Ntherm Nmeas Nsteps
// saveconf. The lattice is t-sharded: ranks_x must be 1 and ranks_t == P.
// Nx/Nt are runtime arguments (the reference's compile-time NS/NT). The
// reference seeds rand() from the clock; here every draw is counter-based
// from `seed` (default: the clock), identical on all ranks. --even-odd uses
// the even-odd preconditioned pseudofermion action (same gauge distribution,
// one half-lattice CG per force; one rank).
//
// Output: the reference's banner and result lines on stdout and its
// 2D_U1_<Nx>x<Nt>_m0<m0>_SimData.txt file; with saveconf = 1 the
// configurations as 2D_U1_Ns<Nx>_Nt<Nt>_b<beta>_m<m0>_<i>.ctxt (28-B records).
#include <mpi.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "sm_hip.h"

namespace {

void die(const char *what) {
    std::cerr << "sm_hmc: " << what << ": " << sm_last_error() << std::endl;
    MPI_Abort(MPI_COMM_WORLD, 1);
}

// include/variables.h:197-203: fixed, 4 decimals, decimal point removed.
std::string format(double number) {
    std::ostringstream oss;
    oss << std::fixed << std::setprecision(4) << number;
    std::string str = oss.str();
    str.erase(str.find('.'), 1);
    return str;
}

}  // namespace

int main(int argc, char **argv) {
    MPI_Init(&argc, &argv);
    int size = 1, rank = 0;
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    int even_odd = 0, npos = 0;
    const char *pos[3] = {nullptr, nullptr, nullptr};
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--even-odd")) even_odd = 1;
        else if (npos < 3) pos[npos++] = argv[i];
    }
    if (npos < 2) {
        if (rank == 0) std::cerr << "usage: sm_hmc <Nx> <Nt> [seed] [--even-odd] < params" << std::endl;
        MPI_Finalize();
        return 2;
    }
    const int Nx = atoi(pos[0]), Nt = atoi(pos[1]);
    unsigned long long seed = npos > 2 ? strtoull(pos[2], nullptr, 10) : (unsigned long long)time(nullptr);
    MPI_Bcast(&seed, 1, MPI_UNSIGNED_LONG_LONG, 0, MPI_COMM_WORLD);

    int ranks_x = 1, ranks_t = 1, MD_steps = 0, Ntherm = 0, Nmeas = 0, Nsteps = 0, saveconf = 0;
    double m0 = 0, trajectory_length = 0, beta = 0;
    const int max_iter = 10000;  // CG::max_iter, src/main.cpp:26
    const double tol = 1e-10;    // CG::tol
    if (rank == 0) {
        std::cerr << "  -----------------------------" << std::endl;
        std::cerr << "|  Two-flavor Schwinger model   |" << std::endl;
        std::cerr << "| Hybrid Monte Carlo simulation |" << std::endl;
        std::cerr << "  -----------------------------" << std::endl;
        std::cerr << "Nx " << Nx << " Nt " << Nt << std::endl;
        std::cerr << "ranks_x: " << std::endl;
        std::cin >> ranks_x;
        std::cerr << "ranks_t: " << std::endl;
        std::cin >> ranks_t;
        std::cerr << "m0: " << std::endl;
        std::cin >> m0;
        std::cerr << "Molecular dynamics steps: " << std::endl;
        std::cin >> MD_steps;
        std::cerr << "Trajectory length: " << std::endl;
        std::cin >> trajectory_length;
        std::cerr << "beta: " << std::endl;
        std::cin >> beta;
        std::cerr << "Thermalization: " << std::endl;
        std::cin >> Ntherm;
        std::cerr << "Measurements: " << std::endl;
        std::cin >> Nmeas;
        std::cerr << "Step (sweeps between measurements): " << std::endl;
        std::cin >> Nsteps;
        std::cerr << "Save configurations yes/no (1 or 0): " << std::endl;
        std::cin >> saveconf;
        std::cerr << std::endl;
    }
    int ip[7] = {ranks_x, ranks_t, MD_steps, Ntherm, Nmeas, Nsteps, saveconf};
    double dp[3] = {m0, trajectory_length, beta};
    MPI_Bcast(ip, 7, MPI_INT, 0, MPI_COMM_WORLD);
    MPI_Bcast(dp, 3, MPI_DOUBLE, 0, MPI_COMM_WORLD);
    ranks_x = ip[0], ranks_t = ip[1], MD_steps = ip[2], Ntherm = ip[3], Nmeas = ip[4], Nsteps = ip[5], saveconf = ip[6];
    m0 = dp[0], trajectory_length = dp[1], beta = dp[2];
    if (ranks_x != 1 || ranks_t != size) {
        if (rank == 0)
            std::cerr << "sm_hmc shards along t only: use ranks_x = 1 and ranks_t = number of ranks (" << size << ")"
                      << std::endl;
        MPI_Finalize();
        return 1;
    }

    // one GPU per rank: node-local rank modulo the visible devices
    MPI_Comm node;
    int local = 0, ndev = 1;
    MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node);
    MPI_Comm_rank(node, &local);
    MPI_Comm_free(&node);
    if (sm_device_count(&ndev) != SM_OK || ndev < 1) die("no GPU");
    // shards over RCCL, or over the device-initiated peer transport with
    // SM_HMC_TRANSPORT=peer (the region handles all-gathered over MPI)
    const char *te = std::getenv("SM_HMC_TRANSPORT");
    const std::string transport = te ? te : "rccl";
    if (transport != "peer" && transport != "rccl") die("SM_HMC_TRANSPORT must be peer or rccl");
    sm_ctx *ctx = nullptr;
    if (size > 1 && transport == "peer") {
        const int nb = sm_peer_handle_bytes();
        std::vector<char> mine((size_t)nb), all((size_t)nb * size);
        if (sm_create_peer(&ctx, Nx, Nt, size, rank, local % ndev, mine.data(), nb) != SM_OK) die("sm_create_peer");
        MPI_Allgather(mine.data(), nb, MPI_BYTE, all.data(), nb, MPI_BYTE, MPI_COMM_WORLD);
        if (sm_peer_connect(ctx, all.data(), nb) != SM_OK) die("sm_peer_connect");
    } else {
        unsigned char uid[256] = {0};
        if (size > 1) {
            if (rank == 0 && sm_comm_unique_id(uid, sizeof uid) != SM_OK) die("sm_comm_unique_id");
            MPI_Bcast(uid, sizeof uid, MPI_BYTE, 0, MPI_COMM_WORLD);
        }
        if (sm_create(&ctx, Nx, Nt, size, rank, local % ndev, size > 1 ? uid : nullptr) != SM_OK) die("sm_create");
    }

    std::string start_time_str;
    if (rank == 0) {
        const std::time_t now_c = std::chrono::system_clock::to_time_t(std::chrono::system_clock::now());
        std::ostringstream tss;
        tss << std::put_time(std::localtime(&now_c), "%Y-%m-%d %H:%M:%S");
        start_time_str = tss.str();
    }
    std::ostringstream NameData;
    NameData << "2D_U1_" << Nx << "x" << Nt << "_m0";
    {
        std::ostringstream m0_stream;
        m0_stream << std::setprecision(17) << m0;
        NameData << m0_stream.str();
    }
    NameData << "_SimData.txt";
    const char *hostname = std::getenv("HOSTNAME");
    std::ofstream Datfile;
    if (rank == 0) {
        Datfile.open(NameData.str());
        Datfile << "#Date and time\n" << start_time_str << "\n";
        Datfile << "#Host\n" << (hostname ? hostname : "unknown") << "\n";
        Datfile << "#Nx      #Nt\n" << std::setw(10) << Nx << std::setw(10) << Nt << "\n";
        Datfile << "#ranks_x     #ranks_t     #ranks\n";
        Datfile << std::setw(15) << ranks_x << std::setw(15) << ranks_t << std::setw(15) << size << "\n";
        Datfile << "#beta                        #Ntherm     #Nmeas     #Nsteps\n";
        Datfile << std::setw(30) << std::setprecision(17) << beta << std::setw(11) << Ntherm << std::setw(11) << Nmeas
                << std::setw(11) << Nsteps << "\n";
        Datfile << "#trajectory_length     #MD_steps\n";
        Datfile << std::setw(30) << std::setprecision(17) << trajectory_length << std::setw(30) << MD_steps << "\n";
        Datfile << "#CG max iterations     #CG relative tolerance\n";
        Datfile << std::setw(30) << max_iter << std::setw(30) << std::setprecision(17) << tol << "\n";
        Datfile << "#m0\n" << std::setw(30) << std::setprecision(17) << m0 << "\n";
        Datfile.close();
        // One-line run summary (key=value, for logs); the SimData file above
        // is the interface other tools read.
        long V = 0;
        sm_local_sites(ctx, &V, nullptr, nullptr, nullptr);
        std::cout << "sm_hmc run: lattice=" << Nx << "x" << Nt << " m0=" << m0 << " kappa=" << 1 / (2 * (m0 + 2))
                  << " beta=" << beta << " therm=" << Ntherm << " meas=" << Nmeas << " skip=" << Nsteps
                  << " tau=" << trajectory_length << " md_steps=" << MD_steps
                  << " eps=" << trajectory_length / MD_steps << " cg_max_iter=" << max_iter << " cg_tol=" << tol
                  << " ranks=" << ranks_x << "x" << ranks_t << " sites_per_rank=" << V
                  << " action=" << (even_odd ? "even-odd" : "full") << " seed=" << seed
                  << " host=" << (hostname ? hostname : "unknown") << " start=" << start_time_str << std::endl;
    }

    sm_hmc_params p;
    p.m0 = m0;
    p.beta = beta;
    p.tau = trajectory_length;
    p.md_steps = MD_steps;
    p.cg_tol = tol;
    p.cg_max_iter = max_iter;
    p.seed = seed;
    p.even_odd = even_odd;
    std::ostringstream save;
    save << "2D_U1_Ns" << Nx << "_Nt" << Nt << "_b" << format(beta) << "_m" << format(m0);
    const std::string save_prefix = save.str();
    sm_hmc_summary s;
    MPI_Barrier(MPI_COMM_WORLD);
    const double begin = MPI_Wtime();
    if (sm_hmc_run(ctx, &p, 1, 0, Ntherm, Nmeas, Nsteps, saveconf == 1 ? save_prefix.c_str() : nullptr, &s, nullptr,
                   nullptr) != SM_OK)
        die("sm_hmc_run");
    MPI_Barrier(MPI_COMM_WORLD);
    const double end = MPI_Wtime();

    if (rank == 0) {
        // the reference prints accepted/(Nmeas + Nsteps*Nmeas) here and writes
        // accepted/(Nmeas + Nsteps*(Nmeas-1)) to the file (src/main.cpp:162,169)
        const double acc_stdout = s.accepted / ((Nmeas + Nsteps * Nmeas) * 1.0);
        std::cout << "Average plaquette value / volume: Ep = " << s.Ep << " dEp = " << s.dEp << std::endl;
        std::cout << "Average gauge action / volume: gS = " << s.gS << " dgS = " << s.dgS << std::endl;
        std::cout << "Acceptance rate: " << acc_stdout << std::endl;
        std::cout << "Execution time = " << end - begin << " s" << std::endl;
        std::cout << "CG iterations = " << s.cg_iterations << ", CG failures = " << s.cg_failures
                  << ", trajectories = " << s.trajectories << ", CG link bytes/site = " << s.cg_link_bytes
                  << std::endl;
        std::cout << "-------------------------------" << std::endl;
        Datfile.open(NameData.str(), std::ios::app);
        Datfile << "#Ep                           #dEp\n";
        Datfile << std::setw(30) << std::setprecision(17) << s.Ep << std::setw(30) << s.dEp << "\n";
        Datfile << "#gS                           #dgS\n";
        Datfile << std::setw(30) << std::setprecision(17) << s.gS << std::setw(30) << s.dgS << "\n";
        Datfile << "#Acceptance rate\n";
        Datfile << std::setw(30) << std::setprecision(17) << s.acceptance << "\n";
        Datfile << "#Execution time\n";
        Datfile << std::setw(30) << std::setprecision(17) << end - begin;
        Datfile.close();
    }
    sm_destroy(ctx);
    MPI_Finalize();
    return 0;
}
