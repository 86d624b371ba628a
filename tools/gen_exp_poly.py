"""Coefficients of the device exp polynomials (torj_math.hpp exp_fast: degree
11; exp2_node, the Albajar node loop: degree 9, coefficients scaled by ln2^i -- `python tools/gen_exp_poly.py 9 --base2`).

e^r on |r| <= ln2/2 as 1 + r + r^2 q(r), q of degree 9 interpolated at its
Chebyshev nodes in 50-digit arithmetic (near-minimax): degree 11 overall, max
error 0.55 ulp under double Horner evaluation, against 1.51 ulp for the degree
12 Taylor polynomial it replaces.  Prints the coefficients c0..c11 and the error.
"""
import mpmath
import numpy as np
from mpmath import cos, exp, log, mp, mpf, pi

mp.dps = 50
L = log(2) / 2


def fit(deg):
    n = deg - 1
    nodes = [L * cos(pi * (k + mpf(0.5)) / n) for k in range(n)]
    q = lambda r: sum(r ** k / mp.factorial(k + 2) for k in range(60))  # (e^r - 1 - r) / r^2
    A = mpmath.matrix([[nd ** j for j in range(n)] for nd in nodes])
    c = mpmath.lu_solve(A, mpmath.matrix([q(nd) for nd in nodes]))
    return [1.0, 1.0] + [float(c[j]) for j in range(n)]


def max_ulp(co):
    rs = np.linspace(-float(L), float(L), 4001)
    p = np.full_like(rs, co[-1])
    for c in co[-2::-1]:
        p = p * rs + c
    return max(float(abs(mpf(float(v)) - exp(mpf(float(r)))) / exp(mpf(float(r)))) / 2.0 ** -52
               for r, v in zip(rs[::3], p[::3]))


if __name__ == "__main__":
    import sys
    co = fit(int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 11)
    print("max error %.2f ulp" % max_ulp(co))
    for k, v in enumerate(co):
        print(f"c{k} = {v!r}")
    if "--base2" in sys.argv:  # exp2_node: 2^r = e^(r ln2) on |r| <= 1/2, d_k = c_k ln2^k
        for k, v in enumerate(co):
            print(f"d{k} = {float(mpf(v) * log(2) ** k)!r}")
