"""The algebra of the dense engine's non-uniform FFT outputs (csrc/dse_nufft.hip), restated in numpy
and checked against 40-digit direct sums: on np.linspace's grid tau_j = fl(j s),
    sum_a w_a e^{-i lambda_a tau_j} = F_j - i delta_j G_j + O((lambda delta)^2),
    F_j = sum_a w_a e^{-i j theta_a},  G_j = sum_a lambda_a w_a e^{-i j theta_a},
    theta_a = lambda_a s mod 2 pi,  delta_j = tau_j - j s,
with F and G by exponential-of-semicircle spreading (W = 15, beta = 2.30 W) onto M = 2T points, an
M-point FFT and deconvolution by the kernel's Fourier transform (Gauss-Legendre), modes centred at
j - T/2.  The GPU tests (tests/test_gpu_nufft.py) hold the device implementation to the GEMM path and
to the 30 s fixtures."""
import mpmath as mp
import numpy as np

W, BETA_W = 15, 2.30


def _nufft(theta, w, T):
    M = 2 * T
    h = 2 * np.pi / M
    aw = W * h / 2
    beta = BETA_W * W
    half = T // 2
    phi = lambda z: np.where(np.abs(z) < 1, np.exp(beta * (np.sqrt(np.maximum(0.0, 1 - z * z)) - 1)), 0.0)  # noqa: E731
    u = np.zeros(M, complex)
    for a in range(len(theta)):
        ms = np.arange(int(np.ceil((theta[a] - aw) / h)), int(np.floor((theta[a] + aw) / h)) + 1)
        u[ms % M] += w[a] * phi((ms * h - theta[a]) / aw)
    U = np.fft.fft(u)
    k = np.arange(-half, T - half)
    x, gw = np.polynomial.legendre.leggauss(200)
    ph = aw * np.array([np.sum(gw * phi(x) * np.cos(kk * aw * x)) for kk in k])
    return (2 * np.pi / M) * U[k % M] / ph


def test_nufft_with_ulp_correction_matches_direct_sums():
    mp.mp.dps = 40
    rng = np.random.default_rng(7)
    n, T = 64, 256
    s = 30.0 / 19999.0
    tau = np.linspace(0.0, 30.0, 20000)[:T]               # np.linspace's own rounding
    assert tau[1] == s
    lam = rng.uniform(-7e6, 7e6, n)
    w = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    w /= np.sum(np.abs(w))
    delta = np.array([float(mp.mpf(float(tau[j])) - j * mp.mpf(s)) for j in range(T)])
    assert np.max(np.abs(delta)) * 7e6 < 1e-7 and np.max(np.abs(delta)) > 0.0
    theta = np.array([float(mp.fmod(mp.mpf(float(la)) * mp.mpf(s), 2 * mp.pi)) for la in lam]) % (2 * np.pi)
    half = T // 2
    cen = np.array([complex(mp.expj(-(half * mp.mpf(float(la)) * mp.mpf(s)))) for la in lam])
    F = _nufft(theta, w * cen, T)
    G = _nufft(theta, lam * w * cen, T)
    approx = F - 1j * delta * G
    ref = np.array([complex(mp.fsum(mp.mpc(complex(wa)) * mp.expj(-mp.mpf(float(la)) * mp.mpf(float(tau[j])))
                                    for wa, la in zip(w, lam))) for j in range(T)])
    err = float(np.max(np.abs(approx - ref)))
    err_nocorr = float(np.max(np.abs(F - ref)))
    assert err < 1e-13, err                                 # sum |w| = 1
    assert err_nocorr > 10 * err                            # the ulp correction matters
