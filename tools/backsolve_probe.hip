// Dev probe: times k_chol_backsolve (L^T x = y + the camera-trial epilogue)
// on a random well-conditioned factor, with and without the epilogue, and
// checks x against a host back substitution.  Not part of the product.
// Build: tools/backsolve_probe.sh
#include "../structure-from-motion-_amd/csrc/ba.hip"
#include <cstdio>
#include <random>
#include <vector>


int main() {
    const int TB = 16;
    for (int ns : {300, 1200}) {
        const int nT = (ns + TB - 1) / TB, nsp = nT * TB, nc = ns / 6;
        std::mt19937_64 g(ns);
        std::uniform_real_distribution<double> u(-0.1, 0.1);
        std::vector<double> A((size_t)nsp * nsp, 0.0), y(nsp), D(2 * TB * TB, 0.0);
        for (int i = 0; i < nsp; ++i)
            for (int j = 0; j <= i; ++j) {
                const double v = i == j ? 1.0 + std::fabs(u(g)) : u(g);
                A[(size_t)i * nsp + j] = v;
                A[(size_t)j * nsp + i] = v;
            }
        const int k0 = (nT - 1) * TB;
        for (int i = 0; i < TB; ++i)
            for (int j = 0; j <= i; ++j) D[((nT - 1) & 1) * TB * TB + i * TB + j] = A[(size_t)(k0 + i) * nsp + k0 + j];
        for (auto &v : y) v = u(g);
        std::vector<double> x(y);
        for (int i = nsp - 1; i >= 0; --i) {
            double s = x[i];
            for (int m = i + 1; m < nsp; ++m) s -= A[(size_t)m * nsp + i] * x[m];
            x[i] = s / A[(size_t)i * nsp + i];
        }
        std::vector<double> payload((size_t)ns * ns + 3 * ns, 0.5), Rt(12 * nc, 0.0);
        for (int c = 0; c < nc; ++c) Rt[12 * c] = Rt[12 * c + 4] = Rt[12 * c + 8] = 1.0;
        double *dA, *dy, *dD, *dpay, *dRt, *dRt2, *dout, *dlam;
        hipMalloc(&dA, A.size() * 8); hipMalloc(&dy, nsp * 8); hipMalloc(&dD, D.size() * 8);
        hipMalloc(&dpay, payload.size() * 8); hipMalloc(&dRt, Rt.size() * 8); hipMalloc(&dRt2, Rt.size() * 8);
        hipMalloc(&dout, 64); hipMalloc(&dlam, 8);
        const double lam = 1e-3;
        hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
        hipMemcpy(dD, D.data(), D.size() * 8, hipMemcpyHostToDevice);
        hipMemcpy(dpay, payload.data(), payload.size() * 8, hipMemcpyHostToDevice);
        hipMemcpy(dRt, Rt.data(), Rt.size() * 8, hipMemcpyHostToDevice);
        hipMemcpy(dlam, &lam, 8, hipMemcpyHostToDevice);
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        for (int with_ct = 0; with_ct < 2; ++with_ct) {
            CamTrialArgs ct{};
            if (with_ct) ct = CamTrialArgs{nc, ns, dpay, dlam, dRt, dRt2, dout};
            float best = 1e30f;
            for (int r = 0; r < 30; ++r) {
                hipMemcpy(dy, y.data(), nsp * 8, hipMemcpyHostToDevice);
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(k_chol_backsolve<16>, dim3(1), dim3(SOLVE_THREADS), 0, 0, dA, nsp, dy,
                                   dD + ((nT - 1) & 1) * TB * TB, ct, (const int *)nullptr);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                best = std::min(best, ms);
            }
            std::vector<double> xo(nsp);
            hipMemcpy(xo.data(), dy, nsp * 8, hipMemcpyDeviceToHost);
            double ex = 0;
            for (int i = 0; i < nsp; ++i) ex = std::max(ex, std::fabs(xo[i] - x[i]));
            printf("ns=%d nsp=%d cam_trial=%d best_us=%.2f maxerr=%.3e\n", ns, nsp, with_ct, best * 1e3, ex);
        }

    }
    return 0;
}
