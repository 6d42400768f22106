// dwt8_operator.cpp -- the fe=dwt-8 window transform as an explicit 16 x 512 matrix.
//
// WaveletTransform.java:126-137 keeps coefficients 0..15 of the eegdsp 1.0 pyramid of a 512-sample
// window (10-tap Daubechies, 12-decimal taps, periodic extension,
// 512 -> 256 -> ... -> 16, first 16 = a6[0..7] ++ d6[0..7]).  Every level is linear, so
// coefficient r = sum_k M[r][k] x[k]; column k of M is the pyramid applied to the unit vector
// e_k.  The columns are evaluated here in long double (x87, 64-bit mantissa) and rounded once to
// double, so M carries < 1 ulp of error per entry; mfma.hip applies it on the FP64 matrix cores.
//
// M is block-circulant: a window shifted by 64 samples (2^6) shifts a6 and d6 by one position, so
// M[r][k] = M[8 (r >> 3)][(k - 64 (r & 7)) mod 512] and rows 0 (a6[0]) and 8 (d6[0]) define it
// (dwt8_operator_rows; the circulant identity is checked in tests/test_host_native.py).
#include <cstring>
#include <vector>

namespace eegfx {

namespace {
constexpr int kWinN = 512;
// The taps are the reference's double literals (rounded to double first, as Java does).
const double kH[10] = {0.160102397974,  0.603829269797,  0.724308528438, 0.138428145901,
                       -0.242294887066, -0.032244869585, 0.077571493840, -0.006241490213,
                       -0.012580751999, 0.003335725285};
}  // namespace

void dwt8_operator(double* M /* [16][512] */) {
  long double h[10], g[10];
  for (int j = 0; j < 10; ++j) {
    h[j] = kH[j];
    g[j] = (j & 1) ? kH[9 - j] : -kH[9 - j];
  }
  std::vector<long double> x(kWinN), t(kWinN);
  for (int k = 0; k < kWinN; ++k) {
    std::fill(x.begin(), x.end(), 0.0L);
    x[k] = 1.0L;
    for (int n = kWinN; n >= 10; n /= 2) {
      for (int i = 0; i < n / 2; ++i) {
        long double a = 0.0L, d = 0.0L;
        for (int j = 0; j < 10; ++j) {
          const long double v = x[(2 * i + j) % n];
          a += v * h[j];
          d += v * g[j];
        }
        t[i] = a;
        t[i + n / 2] = d;
      }
      std::copy(t.begin(), t.begin() + n, x.begin());
    }
    for (int r = 0; r < 16; ++r) M[r * kWinN + k] = (double)x[r];
  }
}

void dwt8_operator_rows(double* rows /* [2][512] */) {
  std::vector<double> M(16 * kWinN);
  dwt8_operator(M.data());
  std::memcpy(rows, M.data(), sizeof(double) * kWinN);
  std::memcpy(rows + kWinN, M.data() + 8 * kWinN, sizeof(double) * kWinN);
}

}  // namespace eegfx
