// Round-4 gemm4 k-loop schedule A/B (profiles/r4/gemm4_ab_v0-7.txt): every G4Sched variant as
// it was in csrc/kernels/gemm4.hip; the package keeps the two defaults (4, 6).
template <> struct G4Sched<0> {   // DMA in k-step 1, early wait (lead ~0.9 k-tile)
  static constexpr int q0 = 2, qs = 2, b1 = 47, d0 = 64, ds = 2, b2 = 79, vm = 8, p0 = 81, ps = 2;
};
template <> struct G4Sched<1> {   // DMA right after B1 in k-step 0, wait in k-step 1 (lead ~1.25)
  static constexpr int q0 = 0, qs = 2, b1 = 35, d0 = 36, ds = 2, b2 = 88, vm = 16, p0 = 89, ps = 2;
};
template <> struct G4Sched<2> {   // hipBLASLt-like: late wait, dense P reads (lead ~1.4)
  static constexpr int q0 = 0, qs = 2, b1 = 35, d0 = 36, ds = 3, b2 = 104, vm = 16, p0 = 105, ps = 1;
};
template <> struct G4Sched<3> {   // dense Q reads, early DMA
  static constexpr int q0 = 0, qs = 1, b1 = 24, d0 = 25, ds = 2, b2 = 80, vm = 16, p0 = 81, ps = 2;
};
template <> struct G4Sched<4> {   // late wait, DMA spread thin (1 per 4 MFMAs), dense P reads
  static constexpr int q0 = 0, qs = 2, b1 = 35, d0 = 36, ds = 4, b2 = 104, vm = 16, p0 = 105, ps = 1;
};
template <> struct G4Sched<5> {   // dense Q reads, early B1, DMA 1 per 3, late wait
  static constexpr int q0 = 0, qs = 1, b1 = 20, d0 = 21, ds = 3, b2 = 96, vm = 16, p0 = 97, ps = 1;
};
template <> struct G4Sched<6> {   // v4 with the DMA spread over B2 (1 per 6 MFMAs, 12 before it)
  static constexpr int q0 = 0, qs = 2, b1 = 35, d0 = 36, ds = 6, b2 = 104, vm = 12, p0 = 105, ps = 1;
};
template <> struct G4Sched<7> {   // v4 with the DMA 1 per 5 MFMAs (14 before B2)
  static constexpr int q0 = 0, qs = 2, b1 = 35, d0 = 36, ds = 5, b2 = 104, vm = 14, p0 = 105, ps = 1;
};
// bfirst: the weight (B) pieces of a stage go out before the activation (A) pieces -- at decode M
// the activations are L2-resident and the weights stream from HBM, so the HBM loads get the
// longest lead before the barrier that waits for them
template <> struct G4Sched<8> {   // v6, weights first
  static constexpr int q0 = 0, qs = 2, b1 = 35, d0 = 36, ds = 6, b2 = 104, vm = 12, p0 = 105, ps = 1;
  static constexpr bool bfirst = true;
};
template <> struct G4Sched<9> {   // v4, weights first
  static constexpr int q0 = 0, qs = 2, b1 = 35, d0 = 36, ds = 4, b2 = 104, vm = 16, p0 = 105, ps = 1;
  static constexpr bool bfirst = true;
};
