// layout.h -- kernel-side parameter layout for the AIQMC network (N electrons,
// A atoms, two occupied spin channels, default hidden dims).
//
// The host repacks the canonical tree_flatten parameter vector (see
// include/aiqmc.h) into this layout once per aiqmc_set_params; derived
// quantities (row-normalised y coefficients nn.py:449-451, (2Z)^{3/4},
// (2Z)^{1/4} Jastrow.py:95, e-e cusp/alpha tables Jastrow.py:23-41, V_nn)
// are precomputed there in double precision.
#pragma once

namespace aq {

constexpr int NH = 4;    // h-stream width  (hidden_dims[l][0], nn.py:525)
constexpr int NH2 = 4;   // pair-stream width (hidden_dims[l][1])
constexpr int NYW = 6;   // Ynlm-stream width (hidden_dims_Ynlm, nn.py:526)

template <int N, int A>
struct Lay {
  // conv input widths: (nchannels+1)*d1 + nchannels*d2 with 2 channels (nn.py:209-210)
  static constexpr int D0 = 3 * 4 * A + 2 * NH2;   // layer 0
  static constexpr int D1 = 3 * NH + 2 * NH2;      // layers 1,2
  static constexpr int Q0 = D0 / 4, Q1 = D1 / 4;
  static constexpr int DY0 = 4 * A + 2;            // nn.py:220
  // network_blocks.convolu_layer weights [N][D], bias [N][D/4]
  static constexpr int conv_w0 = 0;
  static constexpr int conv_b0 = conv_w0 + N * D0;
  static constexpr int conv_w1 = conv_b0 + N * Q0;
  static constexpr int conv_b1 = conv_w1 + N * D1;
  static constexpr int conv_w2 = conv_b1 + N * Q1;
  static constexpr int conv_b2 = conv_w2 + N * D1;
  // single linear [Q][4], [4]
  static constexpr int sng_w0 = conv_b2 + N * Q1;
  static constexpr int sng_b0 = sng_w0 + Q0 * NH;
  static constexpr int sng_w1 = sng_b0 + NH;
  static constexpr int sng_b1 = sng_w1 + Q1 * NH;
  static constexpr int sng_w2 = sng_b1 + NH;
  static constexpr int sng_b2 = sng_w2 + Q1 * NH;
  // double (pair) linear [4][4], [4], layers 0 and 1
  static constexpr int dbl_w0 = sng_b2 + NH;
  static constexpr int dbl_b0 = dbl_w0 + NH2 * NH2;
  static constexpr int dbl_w1 = dbl_b0 + NH2;
  static constexpr int dbl_b1 = dbl_w1 + NH2 * NH2;
  // Ynlm stream [in][6], [6]
  static constexpr int y_w0 = dbl_b1 + NH2;
  static constexpr int y_b0 = y_w0 + DY0 * NYW;
  static constexpr int y_w1 = y_b0 + NYW;
  static constexpr int y_b1 = y_w1 + NYW * NYW;
  static constexpr int y_w2 = y_b1 + NYW;
  static constexpr int y_b2 = y_w2 + NYW * NYW;
  // orbitals: W[spin][f][col][re,im], b[spin][col][re,im]  (nn.py:447,456)
  static constexpr int orb_w = y_b2 + NYW;
  static constexpr int orb_b = orb_w + 2 * NH * N * 2;
  // normalised y coefficients [6][N]
  static constexpr int wy = orb_b + 2 * N * 2;
  // Jastrow e-e: cusp [N][N] (0.25 par / 0.5 anti / 0 diag), alpha [N][N]
  static constexpr int jee_c = wy + NYW * N;
  static constexpr int jee_a = jee_c + N * N;
  // Jastrow e-n beta [N][A]
  static constexpr int jae_b = jee_a + N * N;
  // envelope per electron: alpha[N], xi[N], beta[N][A], pi[N][A][3], sigma[N][A][3]
  static constexpr int env_alpha = jae_b + N * A;
  static constexpr int env_xi = env_alpha + N;
  static constexpr int env_beta = env_xi + N;
  static constexpr int env_pi = env_beta + N * A;
  static constexpr int env_sigma = env_pi + N * A * 3;
  // system
  static constexpr int atoms = env_sigma + N * A * 3;
  static constexpr int charges = atoms + 3 * A;
  static constexpr int c34 = charges + A;
  static constexpr int c14 = c34 + A;
  static constexpr int vnn = c14 + A;
  static constexpr int total = vnn + 1;   // the parameters proper (per-walker gradients use this many)

  // Lane-order copies for the register-resident h-stream layers (k_walker_rev F4 / B2, lane =
  // 4 electron + unit f), after the parameters proper and 16-byte aligned: what a lane reads of
  // the conv weights, conv biases and single weights is contiguous here (strided by 4 above), so
  // one dwordx4 load fetches four values (round 4: the proposal launch issued 142 vector loads
  // per wave, most of them these weights, with the texture-address unit 62 % busy).
  // conv outputs per layer, padded to whole 16-byte records (8 for A <= 2: Q0 = 3 A + 2)
  static constexpr int XQ = (Q0 > Q1 ? Q0 : Q1) <= 8 ? 8 : ((Q0 > Q1 ? Q0 : Q1) + 3) / 4 * 4;
  // conv-bias record of a lane: its output of each full quad, then the Q mod 4 outputs every lane
  // evaluates (4 for A <= 2)
  static constexpr int CBN(int q) { return q / 4 + q % 4; }
  static constexpr int XB = (CBN(Q0) > CBN(Q1) ? CBN(Q0) : CBN(Q1)) <= 4 ? 4
                            : ((CBN(Q0) > CBN(Q1) ? CBN(Q0) : CBN(Q1)) + 3) / 4 * 4;
  static constexpr int x0 = (total + 3) / 4 * 4;
  // [3][N][4][XQ] conv weights of (electron i, unit f): w[i][4 q + f], q < Q
  static constexpr int xcw(int l) { return x0 + l * N * 4 * XQ; }
  // [3][4][XQ] single-layer weights of unit f: w[q][f]
  static constexpr int xsw(int l) { return xcw(3) + l * 4 * XQ; }
  // [3][XQ][4] single-layer weight rows w[q][0..3] (aligned copy)
  static constexpr int xsr(int l) { return xsw(3) + l * XQ * 4; }
  // [3][N][4][XB] conv biases of (electron i, unit f): b[i][4 s + f] for the Q / 4 full quads s,
  // then b[i][q] for the Q mod 4 outputs every lane evaluates
  static constexpr int xcb(int l) { return xsr(3) + l * N * 4 * XB; }
  static constexpr int total_ext = xcb(3);   // device parameter buffer
  static_assert(Q0 <= XQ && Q1 <= XQ, "conv outputs exceed the padded lane records");
  static_assert(CBN(Q0) <= XB && CBN(Q1) <= XB, "conv bias record");

  // canonical (tree_flatten) parameter count
  static constexpr long canon(int npar, int nanti) {
    return (long)N * (2 + 12 * A)                       // envelope
           + (long)N * A                                // jastrow_ae
           + npar + nanti                               // jastrow_ee
           + (N * Q0 + N * D0) + (NH2 + NH2 * NH2) + (NH + Q0 * NH)   // streams[0]
           + (N * Q1 + N * D1) + (NH2 + NH2 * NH2) + (NH + Q1 * NH)   // streams[1]
           + (N * Q1 + N * D1) + (NH + Q1 * NH)                        // streams[2]
           + (NYW + DY0 * NYW) + 2 * (NYW + NYW * NYW)                 // streams_y
           + 2 * (2 * N + NH * 2 * N)                                  // orbitals
           + NYW * N;                                                  // y
  }
};

// Per-walker cache of the local-energy launch pair (walker_lap.h): written by the
// adjoint pass k_walker_rev<..., PREP>, read by k_walker_lap.
template <int N, int A>
struct LapCache {
  static constexpr int D0 = 4 * A;
  static constexpr int QM = (3 * D0 + 2 * NH2) / 4;   // conv outputs of layer 0 (the widest layer)
  // one block per h-stream layer l at l * layer_n (staged in LDS a layer at a time)
  static constexpr int cn = 0;                        // [N][QM][2]  conv nodes: (1 - c^2) / 4, abar phi''(z) / 16
  static constexpr int sn = cn + N * QM * 2;          // [N][4][2]   single nodes: 1 - s^2, abar phi''(z)
  static constexpr int sd = sn + N * NH * 2;          // [2][N][3][4] sum_{k in G, k != i} dh2[k,i][f] / d(x_i - x_k)_c
  static constexpr int layer_n = (sd + 2 * N * 3 * NH2 + 3) / 4 * 4;
  static constexpr int h0b = 3 * layer_n;             // [N][D0]     adjoint of the layer-0 features
  static constexpr int bm = (h0b + N * D0 + 3) / 4 * 4;   // [N][N][2] B = A^{-1}
  static constexpr int ph = bm + 2 * N * N;           // [N][N][2]   Phi
  static constexpr int qs = ph + 2 * N * N;           // [N][N][4][2] Q_f[r,s] = sum_c W_{s(r)}[f,c] Yt[r,c] B[c,s]
  static constexpr int scal = qs + 8 * N * N;         // [0]         pair-local part of the Laplacian
  // [N][N][pt_n] per ordered pair (k, i), diagonal included: tanh outputs t1[4], t2[4] of the two double
  // layers, so that the first-derivative pass carries only the derivative chain through the pair stream
  static constexpr int pt_n = 8;
  static constexpr int pt = (scal + 4 + 3) / 4 * 4;
  static constexpr int size = (pt + pt_n * N * N + 31) / 32 * 32;
  // 16-byte loads of k_walker_lap rely on these: the pair records (PairT), the Phi row of an even-N
  // electron (ld_vec of 2N values; odd N loads it element-wise) and the staged blocks, from a 128-byte
  // aligned walker record
  static_assert(pt % 4 == 0 && pt_n % 4 == 0 && (N % 2 == 1 || ph % 4 == 0) && qs % 4 == 0 && bm % 4 == 0 &&
                    size % 32 == 0,
                "LapCache blocks must stay 16-byte aligned");
};

}  // namespace aq
