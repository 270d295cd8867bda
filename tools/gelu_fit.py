"""Fit of the bf16-output GELU (irc_common.h gelu_lite2): x * sigmoid(p(x)),
p(x) = x (c1 + c3 x^2 + c5 x^4), weighted minimax against the exact erf GELU
(weight 1 / (|GELU(x)| + 1e-2)) on [-10, 10], evaluated in fp32 as the kernel does
(clamp to [-9, 9] inside p, exp2 with -log2(e) folded into the coefficients).

    python tools/gelu_fit.py          # prints the coefficients and the error figures
"""
import numpy as np
from scipy.optimize import minimize
from scipy.special import erf

L2E = np.log2(np.e)
CL = 9.0


def model(c, x, f=np.float64):
    x = x.astype(f)
    xc = np.clip(x, -CL, CL).astype(f)
    cc = [f(-L2E * ci) for ci in c]
    u = xc * xc
    q = f(0)
    for ci in cc[::-1]:
        q = q * u + ci
    with np.errstate(over="ignore"):
        e = np.exp2((q * xc).astype(np.float64)).astype(f)
    return (x * (f(1) / (f(1) + e))).astype(np.float64)


def main():
    x = np.linspace(-10, 10, 200001)
    g = 0.5 * x * (1 + erf(x / np.sqrt(2)))
    w = 1.0 / (np.abs(g) + 1e-2)
    err = lambda c: np.max(np.abs(model(c, x) - g) * w)  # noqa: E731
    best = None
    c0 = np.array([1.5976, 0.07056, 0.0])
    for _ in range(10):
        start = c0 if best is None else best.x * (1 + 1e-4 * np.random.randn(3))
        r = minimize(err, start, method="Nelder-Mead",
                     options=dict(maxiter=80000, xatol=1e-14, fatol=1e-16))
        if best is None or r.fun < best.fun:
            best = r
    e32 = np.abs(model(best.x, x, np.float32) - g)
    ag = np.abs(g)
    ulp = 2.0 ** (np.floor(np.log2(np.maximum(ag, 1e-30))) - 7)
    print("coefficients", best.x)
    print("folded (-log2 e * c)", [float(np.float32(-L2E * c)) for c in best.x])
    print("max abs error", e32.max())
    print("max error in bf16 ulp: |g| >= 1e-2", (e32 / ulp)[ag >= 1e-2].max(),
          " |g| >= 1e-4", (e32 / ulp)[ag >= 1e-4].max())


if __name__ == "__main__":
    main()
