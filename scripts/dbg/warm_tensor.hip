// debug aid: dieltens_fr / dieltens_wr on the device vs the host for one point
#include <algorithm>
#include <cstdio>
#include "torj_warm.hpp"
using namespace torj;

__global__ void k(double xg, double yg, double anpl, double amu, int lrm, int iwarm, Tensor *out) {
    Tensor T;
    if (iwarm == 3)
        dieltens_fr(xg, yg, anpl, amu, lrm, T);
    else
        dieltens_wr(xg, yg, anpl, amu, lrm, T);
    *out = T;
}

__global__ void ka(double om, double X, double Y, double Na, double Np, double Te, double inv, int mode,
                   int iwarm, double *out) {
    cplx n2;
    out[0] = alpha_warm(om, X, Y, Na, Np, Te, inv, mode, iwarm, &n2);
    out[1] = n2.re, out[2] = n2.im;
}

int main() {
    const double X = 0.6356810078139615, Y = 1.123386636357144, Npar = -0.04727651004849054,
                 Te = 6785.414288396569;
    const double mu = kMe * kC * kC / (Te * kE);
    const int lrm = std::min(larmornumber(Y, Npar, mu), kWarmMaxL);
    Tensor h, g, *d;
    dieltens_fr(X, Y, Npar, mu, lrm, h);
    if (hipMalloc(&d, sizeof(Tensor)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(1), 0, 0, X, Y, Npar, mu, lrm, 3, d);
    if (hipMemcpy(&g, d, sizeof(Tensor), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("lrm %d mu %g\n", lrm, mu);
    for (int l = 0; l < lrm; l++)
        for (int q = 0; q < 6; q++)
            printf("l%d q%d host (% .12e, % .12e) dev (% .12e, % .12e)\n", l, q, h.e[l][q].re,
                   h.e[l][q].im, g.e[l][q].re, g.e[l][q].im);
    printf("e330 host %.12e dev %.12e\n", h.e330.re, g.e330.re);
    double *o, ho[3];
    if (hipMalloc(&o, 3 * sizeof(double)) != hipSuccess) return 1;
    const double om = 2 * kPi * 140e9, Na = 1.1218582593493804;
    for (int mode = 1; mode >= -1; mode -= 2)
        for (int iw = 1; iw <= 3; iw += 2) {
            cplx hn;
            const double ha = alpha_warm(om, X, Y, Na, Npar, Te, 1.0, mode, iw, &hn);
            hipLaunchKernelGGL(ka, dim3(1), dim3(1), 0, 0, om, X, Y, Na, Npar, Te, 1.0, mode, iw, o);
            if (hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost) != hipSuccess) return 1;
            printf("mode %d iwarm %d host a %.10e n2 (%.10e, %.10e) dev a %.10e n2 (%.10e, %.10e)\n",
                   mode, iw, ha, hn.re, hn.im, ho[0], ho[1], ho[2]);
        }
    return 0;
}
