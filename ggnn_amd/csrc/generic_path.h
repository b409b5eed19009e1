// generic_path.h -- host side of the general path (included by ggnn_api.hip
// inside its anonymous namespace, after Cfg / Prof / Zeroer).
//
// Taken for every shape outside the specialised kernels' envelope (hidden
// size not 128 / 256, v > 128; GGNN_GENERIC forces it): the reference's
// default hidden_size 400 (chem_tensorflow.py:95), its buckets up to 198 nodes
// (chem_tensorflow_dense.py:584-585), hidden 64 training.  Every product is a
// k_gemm launch (MFMA, the same precision policy as the fast path), every
// element-wise step a k_generic.h kernel; activations fp32, rows unpadded.
//
// Per timestep t (chem_tensorflow_dense.py:328-333, :391-437, GRUCell):
//   M[g,c]  = h_t[g] W_c + beta_c         z = (g, c) over non-empty tiles
//   X[g]    = sum_c A[g,c] M[g,c]          z = g, terms = g's channel list
//   G       = sigmoid([X, h] Wg + bg)      two terms (X, h) -> (r | u)
//   rh      = r h ;  cc = tanh([X, rh] Wc + bc) ;  h_{t+1} = u h + (1-u) cc
// and the backward of SURVEY.md Appendix A in the same decomposition.
#pragma once

struct GenAdjL {
  size_t Ag, AgT, occ, chl, cgl, cgc, total;
  int vp;
  int nch, gch;  // cgc: every channel's graph list cut into nch chunks of <= gch graphs
  // pair mode (GGNN_SPARSE_PAIRS, k_pairs.h)
  size_t degc, pidx, pcnt, poff, prow, pdeg, ptile, pmask, wtl, wmap, wmask, wst;
  size_t rcnt, roff, rlist;  // reverse gather lists of the backward's dh scatter (k_pair_rev)
  int cap_tiles, zw, chunk;  // product tiles of the pair-row capacity; dW split-K chunks and their tiles
};
GenAdjL gen_adj_layout(const Cfg& c) {
  GenAdjL L;
  size_t o = 0;
  L.vp = (c.vin + 7) & ~7;
  // dW_c = sum over c's graphs of h^T dM: one workgroup per (channel, 128 x
  // 128 output tile) would leave most CUs idle (8 channels x 16 tiles at
  // hidden 400); chunks of the graph list as separate z (fp32 atomics) give
  // about 2048 workgroups
  const int tiles = ((c.H + 127) / 128) * ((c.H + 127) / 128);
  L.nch = std::max(1, std::min(c.b, (2048 + c.C * tiles - 1) / (c.C * tiles)));
  L.gch = (c.b + L.nch - 1) / L.nch;
  L.nch = (c.b + L.gch - 1) / L.gch;
  L.Ag = o;  o += al((size_t)c.b * c.C * c.vin * L.vp * 2);
  L.AgT = o; o += al((size_t)c.b * c.C * c.vin * L.vp * 2);
  L.occ = o; o += al((size_t)c.b * c.C);
  L.chl = o; o += al((size_t)c.b * (c.C + 1) * 4);
  L.cgl = o; o += al((size_t)c.C * (c.b + 1) * 4);
  L.cgc = o; o += al((size_t)c.C * L.nch * (L.gch + 1) * 4);
  L.cap_tiles = (int)(c.pcap / PAIR_TILE);
  L.chunk = pair_chunk(L.cap_tiles);
  L.zw = c.sparse ? L.cap_tiles / L.chunk + c.C : 0;
  if (c.sparse) {
    const size_t N = (size_t)c.b * c.vin;
    L.degc = o;  o += al((size_t)c.C * N * 2);
    L.pidx = o;  o += al((size_t)c.C * N * 4);
    L.pcnt = o;  o += al((size_t)c.C * 4);
    L.poff = o;  o += al((size_t)(c.C + 1) * 4);
    L.prow = o;  o += al((size_t)c.pcap * 4);
    L.pdeg = o;  o += al((size_t)c.pcap * 4);
    L.ptile = o; o += al((size_t)L.cap_tiles * 2 * 4);
    L.pmask = o; o += al((size_t)L.cap_tiles);
    L.wtl = o;   o += al((size_t)L.zw * (1 + L.chunk) * 4);
    L.wmap = o;  o += al((size_t)L.zw * 4);
    L.wmask = o; o += al((size_t)L.zw);
    L.wst = o;   o += al((size_t)(c.C + 1) * 4);  // channel c's dW chunks: z in [wst[c], wst[c+1])
    L.rcnt = o;  o += al(N * 4);
    L.roff = o;  o += al((N + 1) * 4);
    L.rlist = o; o += al((size_t)c.pcap * 4);
  }
  L.total = o;
  return L;
}

struct GenWsL {
  size_t hs, X, G, RH, CC, M, Dl, DXH, DZC, DZG, DRH, GW, gmax, total;
  size_t PY, PZ, PDX;  // pair mode: Y = A h, Z = Y W (dY in the backward), dX gathered, [pcap][H] each
  // (training: Y and dXg keep one slice of cap_tiles * PAIR_TILE rows per
  // timestep, so dW_c = sum_t mask_t (Y_t^T dXg_t) runs as ONE product after
  // the timestep loop; WTL: its term lists, every timestep's tiles of a chunk)
  size_t WTL, pslice;
  // deterministic reductions (round 5): split-K slabs of the weight-gradient
  // products (GemmArgs::slab), the element-wise kernels' bias partials
  // [T][slices][dbg_r | dbg_u | dbc], pair mode's per-tile dbeta partials
  // [T][cap_tiles][H], and k_sum_rows' chunk sums
  size_t SLAB, GBP, GBR, PDB, SUMS, CSP;  // GBR: dbg_r partials of the fused k_gen_bwd2 [T][M/32 * 4][H]
   // CSP: the dense tiles' dbeta column-sum partials [b][C][v/32][H]
  size_t py(int t) const { return PY + (size_t)t * pslice * 4; }
  size_t pdx(int t) const { return PDX + (size_t)t * pslice * 4; }
  size_t nh, ns;  // floats of one [N][H] array; saved-step slots
  size_t hsl(int t) const { return hs + (size_t)t * nh * 4; }
  size_t x(int t) const { return X + (size_t)(t % ns) * nh * 4; }
  // backward: dzc [T][N][H], dzg [T][N][2H] kept per timestep, so the GRU
  // weight gradients run once over all T*N rows after the timestep loop
  size_t dzc(int t) const { return DZC + (size_t)t * nh * 4; }
  size_t dzg(int t) const { return DZG + (size_t)t * nh * 8; }
  size_t g(int t) const { return G + (size_t)(t % ns) * nh * 8; }
  size_t rh(int t) const { return RH + (size_t)(t % ns) * nh * 4; }
  size_t cc(int t) const { return CC + (size_t)(t % ns) * nh * 4; }
};
// rows per slice of the element-wise backward kernels (k_gen_bwd1 / 2): >= 8
// rows each, at most 1024 slices; one bias partial row per slice
long gen_bias_slices(const Cfg& c) {
  const long N = (long)c.b * c.vin;
  return std::max<long>(1, std::min<long>(1024, (N + 7) / 8));
}
// split-K plan of one GRU weight-gradient product with Nn output columns:
// large batches: z = a chunk of rows, the T timesteps as its terms (~512
// workgroups); small: z = (chunk, timestep), ~1024 workgroups
struct GenWgPlan {
  long KC;
  int Z, nterm, zdiv;
};
GenWgPlan gen_wg_plan(const Cfg& c, long Nn) {
  const long N = (long)c.b * c.vin, H = c.H;
  const long tiles = ((H + 127) / 128) * ((Nn + 127) / 128);
  GenWgPlan p;
  if (N / 128 >= 512 / tiles) {
    const long want = std::max<long>(1, 512 / tiles);
    p.KC = std::min<long>(((N + want - 1) / want + 31) & ~31L, (N + 31) & ~31L);
    p.nterm = c.T;
    p.zdiv = 1;
    p.Z = (int)((N + p.KC - 1) / p.KC);
  } else {
    const long zt = std::max<long>(1, 1024 / tiles);
    long KC = ((c.T * N + zt - 1) / zt + 31) & ~31L;
    p.KC = std::min<long>(std::max<long>(KC, 256), (N + 31) & ~31L);
    p.nterm = 0;
    p.zdiv = c.T;
    p.Z = (int)((N + p.KC - 1) / p.KC) * c.T;
  }
  return p;
}
GenAdjL gen_adj_layout(const Cfg& c);
// floats of the largest split-K slab one backward needs
size_t gen_slab_floats(const Cfg& c) {
  const size_t H = c.H;
  size_t m = 0;
  for (long Nn : {(long)H, 2 * (long)H}) m = std::max(m, (size_t)gen_wg_plan(c, Nn).Z * H * Nn);
  const GenAdjL AL = gen_adj_layout(c);
  if (c.sparse) m = std::max(m, (size_t)AL.zw * H * H);
  else if (AL.nch > 1) m = std::max(m, (size_t)c.C * AL.nch * H * H);
  return m;
}

GenWsL gen_ws_layout(const Cfg& c, bool tr) {
  GenWsL L;
  memset(&L, 0, sizeof(L));
  const size_t N = (size_t)c.b * c.vin, H = c.H;
  L.nh = N * H;
  L.ns = tr ? c.T : 1;
  size_t o = 0;
  const size_t a4 = al(N * H * 4);
  L.nh = a4 / 4;  // slot stride (256-byte aligned)
  L.hs = o;  o += a4 * (tr ? c.T + 1 : 2);
  L.X = o;   o += a4 * L.ns;
  L.G = o;   o += 2 * a4 * L.ns;
  L.RH = o;  o += a4 * L.ns;
  L.CC = o;  o += a4 * L.ns;
  if (c.sparse) {
    const size_t cap_rows = (size_t)(c.pcap / PAIR_TILE) * PAIR_TILE;
    const int slices = tr ? c.T : 1;
    L.pslice = cap_rows * H;
    L.PY = o;  o += al(std::max<size_t>((size_t)c.pcap * H, (size_t)slices * L.pslice) * 4);
    L.PZ = o;  o += al((size_t)c.pcap * H * 4);
    if (tr) {
      L.PDX = o; o += al((size_t)slices * L.pslice * 4);
      const int cap_tiles = (int)(c.pcap / PAIR_TILE), ch = pair_chunk(cap_tiles);
      const size_t zw = (size_t)(cap_tiles / ch) + c.C;
      L.WTL = o; o += al(zw * (1 + (size_t)c.T * ch) * 4);
    }
  } else {
    L.M = o;   o += al((size_t)c.b * c.C * c.vin * H * 4);  // M (forward) / dM (backward), indexed by (g, c)
  }
  if (tr) {
    L.Dl = o;  o += a4;
    L.DXH = o; o += 2 * a4;
    L.DZC = o; o += a4 * c.T;
    L.DZG = o; o += 2 * a4 * c.T;
    L.DRH = o; o += a4;
    if (c.ed && !c.sparse) { L.GW = o; o += al((size_t)c.C * H * H * 4); }
    L.gmax = o; o += al(GMAX_BYTES);
    L.SLAB = o; o += al(gen_slab_floats(c) * 4);
    L.GBP = o;  o += al((size_t)c.T * gen_bias_slices(c) * 3 * H * 4);
    L.GBR = o;  o += al((size_t)c.T * ((N + 31) / 32) * 4 * H * 4);
    if (c.sparse) { L.PDB = o; o += al((size_t)c.T * (c.pcap / PAIR_TILE) * H * 4); }
    L.SUMS = o; o += al((size_t)SUM_RCS * (3 * H + c.C * H) * 4);
    if (!c.sparse) { L.CSP = o; o += al((size_t)c.b * c.C * ((c.vin + 31) / 32) * H * 4); }
  }
  L.total = o;
  return L;
}

GemmArgs gg_args() {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.zdiv = 1;
  a.Z = 1;
  a.alpha = 1.0f;
  a.scA = a.scB = 1.0f;
  return a;
}

// k_gemm_ring (k_gemm_ring.h) takes a product when every 16-byte DMA chunk of
// its operands is a whole, aligned piece of one operand row: 16-byte aligned
// bases, the non-unit strides multiples of a chunk (4 fp32 / 8 u16), the
// contiguous extent (K, or the rows of a row-contiguous operand) inside its
// stride.  Everything else (odd hidden sizes, o = 150 head rows, the
// transposed adjacency) runs on k_gemm.
static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
static bool ring_ok(const GemmArgs& a, bool A16, bool AKC, bool BKC) {
  if (A16 && !AKC) return false;
  const long va = A16 ? 8 : 4;
  if (!al16(a.A) || (a.A2 && !al16(a.A2)) || (a.Am2 && !al16(a.Am2)) || !al16(a.B)) return false;
  if (a.sAp % va || a.sAq % va || a.sBp % 4 || a.sBq % 4) return false;
  // k-contiguous fp32 operands: whole chunks up to K (and up to every split-K
  // chunk's end); 16-bit: zeros from K to the next multiple of 8 (the caller's
  // padding)
  const bool kc4 = a.K % 4 == 0 && (a.Ktot == a.K || (a.Ktot % 4 == 0 && a.sKp % 4 == 0));
  if ((AKC && !A16 && !kc4) || (BKC && !kc4)) return false;
  if (AKC) {
    if (a.sAk != 1 || a.sAm % va || (a.M > 1 && a.K > a.sAm)) return false;
  } else {
    const long rows = a.Msplit ? std::max<long>(a.Msplit, a.M - a.Msplit) : a.M;
    if (a.sAm != 1 || a.sAk % 4 || a.Msplit % 4 || (a.K > 1 && rows > a.sAk)) return false;
  }
  if (BKC) {
    if (a.sBk != 1 || a.sBn % 4 || (a.N > 1 && a.K > a.sBn)) return false;
  } else {
    if (a.sBn != 1 || a.sBk % 4 || (a.K > 1 && a.N > a.sBk)) return false;
  }
  return true;
}
// ggnn_dbg_gemm_ex's kernel choice (0 auto, 1 k_gemm, 2 k_gemm_ring or fail);
// thread-local, so a forward / backward on another thread never sees it
static thread_local int g_gemm_force = 0;
// ring depth: 2 slots (64 KiB: two workgroups per CU) -- measured 1.4-2x
// faster than a 4-slot ring (one workgroup per CU) on every probe shape
// (tools/gemm_ring_probe.py): a second workgroup's MFMAs cover one's prologue,
// barriers and epilogue better than deeper prefetch does.  (Round 5: also at
// the 20-sentence batch's small grids, where one might expect the opposite --
// 4 slots for grids under 2 workgroups per CU: prop 0.507 -> 0.541 ms, wgrad
// unchanged; 4 slots for the masked pair dW: wgrad 0.360 -> 0.435 ms.)

// operand layouts: AKC = A[m][k] with k contiguous, else m contiguous;
// BKC = B stored [n][k] (k contiguous), else B[k][n] (n contiguous)
// k_gemm_ks's column split for a product (0: not a k_gemm_ks product): K
// split over the waves for one-z products whose 32-row grid leaves the chip
// mostly idle and walks >= 8 K slices (the GRU products of a 20-sentence
// batch): the narrowest column split whose grid stays within two workgroups
// per CU.  (Not for term-listed tiles: over the pair tiles of a 20-sentence
// batch 32 x 32 tiles measured slower -- prop_fwd 0.226 -> 0.249 ms per step,
// W_c and Y re-read per column block -- and a graph's channel list would hand
// the waves other terms under channel skipping, which must stay bit-identical
// to the dense loop.)
int gg_ks_wn(GemmArgs a, bool A16, bool AKC, bool BKC) {
  if (a.Ktot == 0) a.Ktot = a.K;
  if (g_gemm_force == 1 || !ring_ok(a, A16, AKC, BKC)) return 0;
  const long grid128 = (long)((a.N + 127) / 128) * ((a.M + 127) / 128) * a.Z;
  const bool small = AKC && (a.M <= 64 || grid128 < 128);
  const bool sc = a.scA != 1.0f || a.scB != 1.0f || a.snum;
  const long kslices = (long)((a.K + 31) / 32) * std::max(a.nterm, 1);
  if (A16 || !AKC || sc || a.tgroups > 1 || a.Z != 1 || a.tl) return 0;
  if (g_gemm_force >= 3) return 1 << (g_gemm_force - 3);  // forced: 3 -> WN 1, 4 -> 2, 5 -> 4
  for (int c = 1; c <= 4 && small && kslices >= 8 && g_gemm_force != 2; c *= 2)
    if ((long)((a.M + 31) / 32) * ((a.N + 32 * c - 1) / (32 * c)) <= 512) return c;
  return 0;
}
// the fused r * h output of a gates product (GemmArgs::aux) as its own pass,
// behind the instances whose epilogue does not carry it
inline void gen_rh_after(const GemmArgs& a, hipStream_t s) {
  if (a.aux)
    hipLaunchKernelGGL(k_gen_rh, dim3(grid1d((long)a.M * a.auxN)), dim3(256), 0, s, (const float*)a.D, a.auxin,
                       a.aux, (long)a.M, a.auxN);
  if (a.bout)
    hipLaunchKernelGGL(k_gen_blend, dim3(grid1d((long)(a.M / a.bv) * ((a.bv + 3) / 4) * a.N)), dim3(256), 0, s,
                       a.bu, a.bh, (const float*)a.D, a.bout, (long)a.M, a.N, a.bv, a.bsd, a.bt);
}
template <int PREC>
int gg_launch(GemmArgs a, bool A16, bool AKC, bool BKC, int kind, hipStream_t s) {
  if (a.Z < 1 || a.M < 1 || a.N < 1) return GGNN_OK;
  if (a.Ktot == 0) a.Ktot = a.K;
  if (a.E && a.mode == GG_ADD) return fail(GGNN_EINVAL, "gemm: an E factor with GG_ADD (the epilogue preloads one of them)");
  if (a.aux && (a.E || a.mode != GG_STORE || a.epi != GG_EPI_SIGMOID || a.Z != 1 || a.Nsplit || a.dr.thr ||
                a.sDm != 2L * a.auxN || a.sDn != 1 || a.N != 2 * a.auxN))
    return fail(GGNN_EINVAL, "gemm: the fused r * h output takes the plain [M][2 auxN] gates store only");
  if (a.bout && (a.E || a.mode != GG_STORE || a.epi != GG_EPI_TANH || a.Z != 1 || a.Nsplit || a.dr.thr ||
                 a.sDm != a.N || a.sDn != 1 || a.bv < 1 || a.M % a.bv))
    return fail(GGNN_EINVAL, "gemm: the fused blend takes the plain [M][N] candidate store only");
  if (a.b2dzg && (a.E || a.mode != GG_STORE || a.epi != GG_EPI_NONE || a.dr.thr || a.Nsplit < 1 ||
                  a.N != 2 * a.Nsplit || !a.b2r || !a.b2h || !a.b2dxh || !a.b2part || !gg_ks_wn(a, A16, AKC, BKC)))
    return fail(GGNN_EINVAL, "gemm: the fused d(rh) epilogue takes the [dX1 | d(rh)] product as a k_gemm_ks launch only");
  if (g_gemm_force != 1 && ring_ok(a, A16, AKC, BKC)) {
    // 32-row tiles for products over one small graph's rows (M <= 64, e.g. the
    // per-(graph, channel) products of v = 30 sentence graphs), and for
    // products whose 128-row grid would leave most CUs idle (the GRU products
    // of a 20-sentence batch: M ~ 600 rows -> 5 x 7 tiles); 128 otherwise
    const long grid128 = (long)((a.N + 127) / 128) * ((a.M + 127) / 128) * a.Z;
    const bool small = AKC && (a.M <= 64 || grid128 < 128);
    const int bm = small ? 32 : 128;
    const int tn = (a.N + 127) / 128, tm = (a.M + bm - 1) / bm;
    const long nwg = (long)tn * tm * a.Z;
    if (nwg > 0x7fffffffL) return fail(GGNN_EINVAL, "k_gemm_ring: grid too large");
    const dim3 grid((unsigned)nwg);
    Prof p(kind, s);
    const bool sc = a.scA != 1.0f || a.scB != 1.0f || a.snum;
    // K split over the waves: k_gemm_ks (gg_ks_wn)
    const int wn = gg_ks_wn(a, A16, AKC, BKC);
    if (wn) {
      const int tn32 = (a.N + 32 * wn - 1) / (32 * wn), tm32 = (a.M + 31) / 32;
      const dim3 g32((unsigned)((long)tn32 * tm32));
#define GKS(BKC_, WN_) hipLaunchKernelGGL((k_gemm_ks<PREC, BKC_, false, WN_>), g32, dim3(256), 0, s, a, tm32, tn32)
      if (BKC) {
        if (wn == 1) GKS(true, 1);
        else if (wn == 2) GKS(true, 2);
        else GKS(true, 4);
      } else {
        if (wn == 1) GKS(false, 1);
        else if (wn == 2) GKS(false, 2);
        else GKS(false, 4);
      }
#undef GKS
      return GGNN_OK;
    }
    // the ring instances keep their epilogue: r * h by its own pass after them
    const GemmArgs rh = a;
    a.aux = nullptr;
    a.bout = nullptr;
    if (g_gemm_force >= 3) return fail(GGNN_EINVAL, "k_gemm_ks: fp32 k-contiguous A, one z, unscaled operands only");
    // plain stores with no epilogue options (the weight-gradient split-K
    // products, the pair products): the instance without the general
    // epilogue, whose registers (256 VGPRs + 85 AGPRs at 128-row tiles) held
    // one workgroup per CU
    const bool lean = a.epi == GG_EPI_NONE && !a.dr.thr && !a.Nsplit &&
                      (a.mode == GG_STORE || (a.mode == GG_ATOMIC && a.slab));
    if (a.slab && !lean && !A16 && !small && a.tgroups <= 1)
      return fail(GGNN_EINVAL, "k_gemm_ring: split-K slab partials with epilogue options (128-row tiles store slabs lean only)");
#define GGR1(A16_, AKC_, BKC_, BM_)                                                                          \
  do {                                                                                                       \
    if (lean && !A16_) {                                                                                     \
      if (sc) hipLaunchKernelGGL((k_gemm_ring<PREC, false, AKC_, BKC_, true, 2, BM_, false, true>), grid, dim3(256), 0, s, a, tm, tn); \
      else hipLaunchKernelGGL((k_gemm_ring<PREC, false, AKC_, BKC_, false, 2, BM_, false, true>), grid, dim3(256), 0, s, a, tm, tn); \
    } else if (sc) hipLaunchKernelGGL((k_gemm_ring<PREC, A16_, AKC_, BKC_, true, 2, BM_>), grid, dim3(256), 0, s, a, tm, tn);  \
    else hipLaunchKernelGGL((k_gemm_ring<PREC, A16_, AKC_, BKC_, false, 2, BM_>), grid, dim3(256), 0, s, a, tm, tn);    \
  } while (0)
#define GGR(A16_, AKC_, BKC_)              \
  do {                                     \
    if (small) GGR1(A16_, AKC_, BKC_, 32);  \
    else GGR1(A16_, AKC_, BKC_, 128);       \
  } while (0)
    if (A16 && !BKC) GGR(true, true, false);
    else if (A16) return fail(GGNN_EINVAL, "k_gemm_ring: operand layout combination not compiled");
    else if (AKC && !BKC) GGR(false, true, false);
    else if (AKC && BKC) GGR(false, true, true);
    else if (!AKC && !BKC && a.tgroups > 1) {
      if (a.dr.thr && !a.mbits) return fail(GGNN_EINVAL, "k_gemm_ring: masked term groups need the mask bits (the pack's)");
      // (whole z's round-robin over the XCDs: the grid covers a multiple of 8 z's)
      const dim3 grid((unsigned)((long)tn * tm * ((a.Z + 7) / 8) * 8));
      // (a 4-slot ring, three slices in flight at one workgroup per CU, measured
      // slower for the weight-gradient products: 1.37 -> 1.72 ms at the
      // reference configuration)
      if (sc) hipLaunchKernelGGL((k_gemm_ring<PREC, false, false, false, true, 2, 128, true>), grid, dim3(256), 0, s, a, tm, tn);
      else hipLaunchKernelGGL((k_gemm_ring<PREC, false, false, false, false, 2, 128, true>), grid, dim3(256), 0, s, a, tm, tn);
    } else if (!AKC && !BKC) GGR1(false, false, false, 128);
    else return fail(GGNN_EINVAL, "k_gemm_ring: operand layout combination not compiled");
#undef GGR
#undef GGR1
    gen_rh_after(rh, s);
    return GGNN_OK;
  }
  if (a.tgroups > 1) return fail(GGNN_EUNSUP, "per-timestep term groups need the ring kernel (16-byte aligned operands)");
  // 64 x 64 block tiles: measured faster than the 128 x 64 / 128 x 128
  // variants of k_gemm on every shape tried (tools/gemm_probe.py: 4096^3, the
  // heads' 32768 x {150, 512} x {512, 150, 256}, a per-graph 128 x 256 x 256):
  // the bigger tiles lose more to occupancy than they save in operand
  // conversion per MFMA
  const dim3 grid((unsigned)((a.N + 63) / 64), (unsigned)((a.M + 63) / 64), (unsigned)std::min(a.Z, 65535));
  Prof p(kind, s);  // (kind < 0: no record, the caller's own Prof scope covers it)
#define GGL(A16_, AKC_, BKC_) hipLaunchKernelGGL((k_gemm<PREC, A16_, AKC_, BKC_, 1, 1>), grid, dim3(256), 0, s, a)
  if (A16 && AKC && !BKC) GGL(true, true, false);
  else if (A16 && !AKC && !BKC) GGL(true, false, false);
  else if (!A16 && AKC && !BKC) GGL(false, true, false);
  else if (!A16 && AKC && BKC) GGL(false, true, true);
  else if (!A16 && !AKC && !BKC) GGL(false, false, false);
  else return fail(GGNN_EINVAL, "k_gemm: operand layout combination not compiled");
#undef GGL
  gen_rh_after(a, s);
  return GGNN_OK;
}

// ---------------------------------------------------------------- adjacency
int gen_set_adjacency(const Cfg& c, void* adj, const float* A, hipStream_t s) {
  const GenAdjL L = gen_adj_layout(c);
  Prof p(K_ADJ, s);
  if (c.prec == PREC_BF16)
    hipLaunchKernelGGL(k_gen_adj<false>, dim3((unsigned)(c.b * c.C)), dim3(256), 0, s, A, c.vin, L.vp,
                       P<u16>(adj, L.Ag), P<u16>(adj, L.AgT), P<unsigned char>(adj, L.occ));
  else
    hipLaunchKernelGGL(k_gen_adj<true>, dim3((unsigned)(c.b * c.C)), dim3(256), 0, s, A, c.vin, L.vp,
                       P<u16>(adj, L.Ag), P<u16>(adj, L.AgT), P<unsigned char>(adj, L.occ));
  return GGNN_OK;
}
int gen_set_adjacency_edges(const Cfg& c, void* adj, const int32_t* edges, const int32_t* goff, int64_t ne, int E,
                            hipStream_t s) {
  const GenAdjL L = gen_adj_layout(c);
  Prof p(K_ADJ, s);
  // every buffer this staging clears, in one launch (prow / pdeg are read
  // only by k_pair_fill below)
  FillSet fs;
  fs.add(P<u16>(adj, L.Ag), 0, (size_t)c.b * c.C * c.vin * L.vp * 2);
  fs.add(P<u16>(adj, L.AgT), 0, (size_t)c.b * c.C * c.vin * L.vp * 2);
  fs.add(P<unsigned char>(adj, L.occ), 0, (size_t)c.b * c.C);
  if (c.sparse) {
    fs.add(P<int>(adj, L.prow), 0xFF, (size_t)c.pcap * 4);
    fs.add(P<float>(adj, L.pdeg), 0, (size_t)c.pcap * 4);
  }
  fs.launch(s);
  if (ne > 0)
    hipLaunchKernelGGL(k_gen_adj_edges, dim3((unsigned)std::min(c.b, 4096)), dim3(256), 0, s, edges, goff, c.b, c.vin,
                       L.vp, E, c.prec != PREC_BF16 ? 1 : 0, P<u16>(adj, L.Ag), P<u16>(adj, L.AgT),
                       P<unsigned char>(adj, L.occ));
  if (c.sparse) {
    // pair rows grouped by channel (k_pairs.h S1-S4)
    const long N = (long)c.b * c.vin;
    hipLaunchKernelGGL(k_pair_degree, dim3((unsigned)(c.b * c.C)), dim3(256), 0, s, P<const u16>(adj, L.Ag),
                       P<const unsigned char>(adj, L.occ), c.b, c.C, c.vin, L.vp, P<u16>(adj, L.degc));
    hipLaunchKernelGGL(k_pair_scan, dim3((unsigned)c.C), dim3(1024), 0, s, P<const u16>(adj, L.degc), N,
                       P<int>(adj, L.pidx), P<int>(adj, L.pcnt));
    hipLaunchKernelGGL(k_pair_layout, dim3(1), dim3(1024), 0, s, P<const int>(adj, L.pcnt), c.C, L.cap_tiles, L.zw,
                       L.chunk, P<int>(adj, L.poff), P<int>(adj, L.ptile), P<unsigned char>(adj, L.pmask), P<int>(adj, L.wtl),
                       P<int>(adj, L.wmap), P<unsigned char>(adj, L.wmask), P<int>(adj, L.wst));
    hipLaunchKernelGGL(k_pair_fill, dim3(grid1d((long)c.C * N)), dim3(256), 0, s, P<const u16>(adj, L.degc),
                       P<int>(adj, L.pidx), P<const int>(adj, L.poff), N, (long)c.C * N, (int)c.pcap,
                       P<int>(adj, L.prow), P<float>(adj, L.pdeg));
  }
  return GGNN_OK;
}
// pair mode, the backward's reverse gather lists (k_pair_rev, S5): built by
// the backward that needs them, so an evaluation batch never pays for them
void gen_pairs_rev(const Cfg& c, void* adj, hipStream_t s) {
  const GenAdjL L = gen_adj_layout(c);
  const long N = (long)c.b * c.vin;
  const unsigned rg = (unsigned)std::min<long>((N + 3) / 4, 16384);
  hipLaunchKernelGGL(k_pair_rev<false>, dim3(rg), dim3(256), 0, s, P<const u16>(adj, L.AgT),
                     P<const unsigned char>(adj, L.occ), P<const int>(adj, L.pidx), c.b, c.vin, L.vp, c.C,
                     P<int>(adj, L.rcnt), (const int*)nullptr, (int*)nullptr, (int)c.pcap);
  hipLaunchKernelGGL(k_pair_rev_scan, dim3(1), dim3(1024), 0, s, P<const int>(adj, L.rcnt), N, P<int>(adj, L.roff));
  hipLaunchKernelGGL(k_pair_rev<true>, dim3(rg), dim3(256), 0, s, P<const u16>(adj, L.AgT),
                     P<const unsigned char>(adj, L.occ), P<const int>(adj, L.pidx), c.b, c.vin, L.vp, c.C,
                     (int*)nullptr, P<const int>(adj, L.roff), P<int>(adj, L.rlist), (int)c.pcap);
}

// pair mode, Y = A h over the pair rows (forward F1; recomputed in the backward)
void gen_pairs_y(const Cfg& c, const GenAdjL& AL, const void* adj, const float* h, float* Y, hipStream_t s) {
  // (rows of whole tiles only: a partial tile past cap_tiles holds no pair)
  const int rows = AL.cap_tiles * PAIR_TILE;
  const unsigned grid = (unsigned)std::min<long>((rows + 3) / 4, 16384);
  hipLaunchKernelGGL(k_pair_gather_y, dim3(grid), dim3(256), 0, s, P<const u16>(adj, AL.Ag), P<const int>(adj, AL.prow),
                     P<const int>(adj, AL.ptile), P<const unsigned char>(adj, AL.pmask), h, Y, c.C, c.vin, AL.vp, c.H,
                     rows);
}
// the per-tile product Z = A_op W_c (forward: A_op = Y, B = W; backward: A_op =
// dXg, B = W^T): z = 32-row tile, its channel from the one-entry term list
template <int PREC>
int gen_pairs_product(const Cfg& c, const GenAdjL& AL, const void* adj, const float* Aop, const float* W, bool wt,
                      float* D, int kind, hipStream_t s) {
  const long H = c.H;
  GemmArgs z = gg_args();
  z.A = Aop; z.sAp = PAIR_TILE * H; z.sAm = H; z.sAk = 1;
  z.B = W; z.sBq = H * H;
  if (wt) { z.sBk = 1; z.sBn = H; } else { z.sBk = H; z.sBn = 1; }
  z.D = D; z.sDz = PAIR_TILE * H; z.sDm = H; z.sDn = 1;
  z.tl = P<const int>(adj, AL.ptile); z.ts = 2; z.zmask = P<const unsigned char>(adj, AL.pmask);
  z.Z = AL.cap_tiles; z.M = PAIR_TILE; z.N = (int)H; z.K = (int)H;
#ifdef GGNN_TS
  z.tsprobe = wt ? 4 : 3;
#endif
  return gg_launch<PREC>(z, false, true, wt, kind, s);
}
// channel lists of the staged batch (per graph, per channel); rebuilt by every
// forward so that GGNN_DENSE_CHANNELS can be chosen per call
void gen_lists(const Cfg& c, void* adj, hipStream_t s) {
  const GenAdjL L = gen_adj_layout(c);
  const int n = c.b + c.C;
  hipLaunchKernelGGL(k_gen_lists, dim3((n + 3) / 4), dim3(256), 0, s, P<const unsigned char>(adj, L.occ), c.b,
                     c.C, (c.flags & GGNN_DENSE_CHANNELS) ? 1 : 0, P<int>(adj, L.chl), P<int>(adj, L.cgl),
                     P<int>(adj, L.cgc), L.nch, L.gch);
}

// -------------------------------------------------------------------- forward
template <int PREC>
int gen_forward(const Cfg& c, const void* pack, void* adj, void* ws, bool tr, const float* h0, float* hT,
                hipStream_t s) {
  const GenAdjL AL = gen_adj_layout(c);
  const PackL PL = pack_layout(c);
  const GenWsL L = gen_ws_layout(c, tr);
  const long N = (long)c.b * c.vin, H = c.H, v = c.vin, C = c.C;
  const bool dense_ch = (c.flags & GGNN_DENSE_CHANNELS) != 0;
  gen_lists(c, adj, s);
  {
    Prof p(K_IO, s);
    copy_async(P<float>(ws, L.hsl(0)), h0, N * H, s);
  }
  const float* beta = (c.flags & GGNN_USE_EDGE_BIAS) ? P<float>(pack, PL.beta) : nullptr;
  for (int t = 0; t < c.T; ++t) {
    const size_t hin = tr ? L.hsl(t) : L.hsl(t & 1);
    float* hout = (t + 1 == c.T) ? hT : P<float>(ws, tr ? L.hsl(t + 1) : L.hsl((t + 1) & 1));
    if (c.sparse) {
      // pair mode (k_pairs.h): Y = A h, Z = Y W_c per 32-row tile, X = the
      // row's sum of Z + deg beta
      // (training: Y_t into timestep t's slice, kept for the backward's dW
      // product instead of regathered there)
      float* PY = P<float>(ws, tr ? L.py(t) : L.PY);
      float* PZ = P<float>(ws, L.PZ);
      {
        Prof p(K_PROP_FWD, s);
        gen_pairs_y(c, AL, adj, P<const float>(ws, hin), PY, s);
      }
      if (int e = gen_pairs_product<PREC>(c, AL, adj, PY, P<float>(pack, PL.gw(c.ed ? t : 0)), false, PZ, K_PROP_FWD,
                                          s))
        return e;
      {
        Prof p(K_PROP_FWD, s);
        hipLaunchKernelGGL(k_pair_reduce_x, dim3(grid1d(N * (H / 4))), dim3(256), 0, s, P<const int>(adj, AL.pidx),
                           P<const float>(adj, AL.pdeg), P<const int>(adj, AL.chl), PZ, beta, P<float>(ws, L.x(t)), N,
                           c.vin, c.C, c.H);
      }
    } else {
    // M[g,c] = h_t[g] W_c + beta_c over the non-empty (g, c) tiles
    GemmArgs m = gg_args();
    m.A = P<float>(ws, hin); m.sAp = v * H; m.sAm = H; m.sAk = 1;
    m.B = P<float>(pack, PL.gw(c.ed ? t : 0)); m.sBq = H * H; m.sBk = H; m.sBn = 1;
    m.D = P<float>(ws, L.M); m.sDz = v * H; m.sDm = H; m.sDn = 1;
    m.bias = beta; m.sbq = H;
    m.zdiv = (int)C; m.Z = (int)(c.b * C); m.zmask = dense_ch ? nullptr : P<unsigned char>(adj, AL.occ);
    m.M = (int)v; m.N = (int)H; m.K = (int)H;
    if (int e = gg_launch<PREC>(m, false, true, false, K_PROP_FWD, s)) return e;
    // X[g] = sum over g's channels of A[g,c] M[g,c]
    GemmArgs x = gg_args();
    x.A = P<u16>(adj, AL.Ag); x.sAp = C * v * AL.vp; x.sAq = v * AL.vp; x.sAm = AL.vp; x.sAk = 1;
    x.B = P<float>(ws, L.M); x.sBp = C * v * H; x.sBq = v * H; x.sBk = H; x.sBn = 1;
    x.D = P<float>(ws, L.x(t)); x.sDz = v * H; x.sDm = H; x.sDn = 1;
    x.tl = P<int>(adj, AL.chl); x.ts = C + 1;
    x.Z = c.b; x.M = (int)v; x.N = (int)H; x.K = (int)v;
    if (int e = gg_launch<PREC>(x, true, true, false, K_PROP_FWD, s)) return e;
    }
    // gates = sigmoid([X, h] Wg + bg)
    GemmArgs gt = gg_args();
    gt.A = P<float>(ws, L.x(t)); gt.sAq = ((long)hin - (long)L.x(t)) / 4; gt.sAm = H; gt.sAk = 1;
    gt.B = P<float>(pack, PL.gWg); gt.sBq = H * 2 * H; gt.sBk = 2 * H; gt.sBn = 1;
    gt.D = P<float>(ws, L.g(t)); gt.sDm = 2 * H; gt.sDn = 1;
    gt.bias = P<float>(pack, PL.bg);
    gt.nterm = 2;
    gt.M = (int)N; gt.N = (int)(2 * H); gt.K = (int)H; gt.epi = GG_EPI_SIGMOID;
    gt.aux = P<float>(ws, L.rh(t)); gt.auxin = P<const float>(ws, hin); gt.auxN = (int)H;  // + r h
    if (int e = gg_launch<PREC>(gt, false, true, false, K_GRU_FWD, s)) return e;
    // cc = tanh([X, r h] Wc + bc)
    GemmArgs cd = gg_args();
    cd.A = P<float>(ws, L.x(t)); cd.sAq = ((long)L.rh(t) - (long)L.x(t)) / 4; cd.sAm = H; cd.sAk = 1;
    cd.B = P<float>(pack, PL.gWc); cd.sBq = H * H; cd.sBk = H; cd.sBn = 1;
    cd.D = P<float>(ws, L.cc(t)); cd.sDm = H; cd.sDn = 1;
    cd.bias = P<float>(pack, PL.bc);
    cd.nterm = 2;
    cd.M = (int)N; cd.N = (int)H; cd.K = (int)H; cd.epi = GG_EPI_TANH;
    // + h' = u h + (1 - u) c and the state dropout
    cd.bout = hout; cd.bh = P<const float>(ws, hin); cd.bu = P<const float>(ws, L.g(t));
    cd.bv = (int)c.vin; cd.bt = t; cd.bsd = c.sdrop;
    if (int e = gg_launch<PREC>(cd, false, true, false, K_GRU_FWD, s)) return e;
  }
  LAUNCHCHK();
  return GGNN_OK;
}

// ------------------------------------------------------------------- backward
template <int PREC>
int gen_backward(const Cfg& c, const void* pack, void* adj, void* ws, const float* dhT, float* dh0, float* dW,
                 float* dbeta, float* dWg, float* dbg, float* dWc, float* dbc, hipStream_t s) {
  const GenAdjL AL = gen_adj_layout(c);
  const PackL PL = pack_layout(c);
  const GenWsL L = gen_ws_layout(c, true);
  const long N = (long)c.b * c.vin, H = c.H, v = c.vin, C = c.C;
  const bool use_bias = (c.flags & GGNN_USE_EDGE_BIAS) != 0;
  const bool dense_ch = (c.flags & GGNN_DENSE_CHANNELS) != 0;
  {
    // the GRU weight and bias gradients and, in pair mode, dW and dbeta are
    // stored whole by the fixed-order reductions (§5.1); the dense tiles add
    // dW over the timesteps and dbeta from the column-sum partials
    Prof p(K_IO, s);
    if (!c.sparse) {
      Zeroer z(s);
      z.add(dW, C * H * H);
      if (use_bias) z.add(dbeta, C * H);
    }
  }
  const uint32_t* gmax = P<const uint32_t>(ws, L.gmax);
  float* DXH = P<float>(ws, L.DXH);
  float* DRH = P<float>(ws, L.DRH);
  float* dM = P<float>(ws, L.M);
  {
    Prof p(K_IO, s);
    absmax(dhT, N * H, P<uint32_t>(ws, L.gmax), s);
  }
  if (c.sparse) {
    Prof p(K_PROP_BWD, s);
    gen_pairs_rev(c, adj, s);
  }
  // The weight gradients take single f16 operands in the fp32-parity mode, as
  // the fast path's k_wgrad256 does (measured <= 3.7e-4 normalised against
  // float64; the dh / dX chain keeps the split limbs): a third of the MFMAs
  constexpr int WPREC = Prec<PREC>::split ? PREC_F16 : PREC;
  // k_gen_bwd2 fused into the d(rh) product's epilogue when that product is a
  // k_gemm_ks launch (the small batches), with gbr_rows dbg_r partial rows a
  // timestep
  int gbr_rows = 0;
  {
    GemmArgs q = gg_args();
    q.A = P<float>(ws, L.dzc(0)); q.B = P<float>(pack, PL.gWc); q.D = DXH;
    q.sAm = H; q.sAk = 1; q.sBk = 1; q.sBn = H; q.sDm = 2 * H; q.sDn = 1; q.sD2m = H; q.Nsplit = (int)H;
    q.M = (int)N; q.N = (int)(2 * H); q.K = (int)H;
    const int wn = gg_ks_wn(q, false, true, true);
    if (wn) gbr_rows = (int)((N + 31) / 32) * (4 / wn);
  }
  const bool fuse2 = gbr_rows > 0;
  for (int t = c.T - 1; t >= 0; --t) {
    const float* ht = P<float>(ws, L.hsl(t));
    float* DZC = P<float>(ws, L.dzc(t));
    float* DZG = P<float>(ws, L.dzg(t));
    const float* G = P<float>(ws, L.g(t));
    // (row slices of the element-wise kernels: >= 8 rows each, at most 1024 slices; one bias
    // atomic per column per slice.  A small batch -- 20 sentences, N ~ 560 rows -- needs the
    // short slices: a thread walks its slice's rows one after another)
    const dim3 ewg((unsigned)((H + 255) / 256), (unsigned)gen_bias_slices(c));
    float* gbp = P<float>(ws, L.GBP) + (size_t)t * ewg.y * 3 * H;  // this timestep's bias partial rows
    {
      Prof p(K_GRU_BWD, s);
      // delta of step t: S * dL/dh_T at the last step, else the dh step t + 1
      // left in DXH's second half; the state dropout of timestep t
      const bool last_t = t == c.T - 1;
      hipLaunchKernelGGL(k_gen_bwd1, ewg, dim3(256), 0, s, last_t ? dhT : DXH + H, last_t ? H : 2 * H,
                         last_t ? gmax : (const uint32_t*)nullptr, c.sdrop, t, (int)c.vin, G, ht,
                         P<const float>(ws, L.cc(t)), DZC, DZG, DXH, N, c.H, gbp);
    }
    // [dX1 | d(rh)] = dzc Wc^T  (Wc [2H][H]: B(k, n) = Wc[n][k]), one launch
    // over both halves: columns n >= H go to d(rh) (a separate [N][H] buffer)
    {
      GemmArgs a = gg_args();
      a.A = DZC; a.sAm = H; a.sAk = 1;
      a.B = P<float>(pack, PL.gWc); a.sBk = 1; a.sBn = H;
      a.D = DXH; a.sDm = 2 * H; a.sDn = 1;
      a.D2 = DRH; a.Nsplit = (int)H; a.sD2m = H;
      a.M = (int)N; a.N = (int)(2 * H); a.K = (int)H;
      if (fuse2) {
        // + k_gen_bwd2 in k_gemm_ks's epilogue; dbg_r partials per (32-row
        // tile, K-slice wave) in GBR
        a.b2r = G; a.b2h = ht; a.b2dzg = DZG; a.b2dxh = DXH;
        a.b2part = P<float>(ws, L.GBR) + (size_t)t * gbr_rows * H;
      }
      if (int e = gg_launch<PREC>(a, false, true, true, K_GRU_BWD, s)) return e;
    }
    if (!fuse2) {
      Prof p(K_GRU_BWD, s);
      hipLaunchKernelGGL(k_gen_bwd2, ewg, dim3(256), 0, s, DRH, G, ht, DZG, DXH, N, c.H, gbp);
    }
    // [dX | dh] += dzg Wg^T
    {
      GemmArgs a = gg_args();
      a.A = DZG; a.sAm = 2 * H; a.sAk = 1;
      a.B = P<float>(pack, PL.gWg); a.sBk = 1; a.sBn = 2 * H;
      a.D = DXH; a.sDm = 2 * H; a.sDn = 1; a.mode = GG_ADD;
      a.M = (int)N; a.N = (int)(2 * H); a.K = (int)(2 * H);
      if (int e = gg_launch<PREC>(a, false, true, true, K_GRU_BWD, s)) return e;
    }
    if (c.sparse) {
      // pair mode (k_pairs.h): Y_t as the training forward left it in its
      // slice, dXg = dX of the pair rows, dbeta, dY = dXg W_c^T, dh += A^T dY,
      // dW_c += Y^T dXg
      float* PZ = P<float>(ws, L.PZ);
      float* PDX = P<float>(ws, L.pdx(t));
      {
        Prof p(K_PROP_BWD, s);
        // dXg gathered, with the dbeta partial of every pair tile (one
        // channel's rows): sum of deg * dXg, summed per channel in tile order
        // after the timestep loop
        if (H <= 1024)
          hipLaunchKernelGGL(k_pair_gather_dx_dbeta, dim3((unsigned)AL.cap_tiles), dim3(256), 0, s,
                             P<const int>(adj, AL.prow), P<const unsigned char>(adj, AL.pmask),
                             P<const float>(adj, AL.pdeg), DXH, PDX,
                             use_bias ? P<float>(ws, L.PDB) + (size_t)t * AL.cap_tiles * H : (float*)nullptr, c.H);
        else {
          hipLaunchKernelGGL(k_pair_gather_dx, dim3(grid1d((long)AL.cap_tiles * PAIR_TILE * (H / 4))), dim3(256), 0,
                             s, P<const int>(adj, AL.prow), P<const unsigned char>(adj, AL.pmask), DXH, PDX,
                             AL.cap_tiles * PAIR_TILE, c.H);
          if (use_bias)
            hipLaunchKernelGGL(k_pair_dbeta, dim3((unsigned)((H + 255) / 256), (unsigned)AL.cap_tiles), dim3(256), 0,
                               s, P<const unsigned char>(adj, AL.pmask), P<const float>(adj, AL.pdeg), PDX,
                               P<float>(ws, L.PDB) + (size_t)t * AL.cap_tiles * H, c.H);
        }
      }
      if (int e = gen_pairs_product<PREC>(c, AL, adj, PDX, P<float>(pack, PL.gw(c.ed ? t : 0)), true, PZ, K_PROP_BWD,
                                          s))
        return e;
      {
        Prof p(K_PROP_BWD, s);
        hipLaunchKernelGGL(k_pair_scatter_dh, dim3((unsigned)std::min<long>((N + 3) / 4, 16384)), dim3(256), 0, s,
                           P<const int>(adj, AL.roff), P<const int>(adj, AL.rlist), PZ, DXH, N, c.H);
      }
      // (dW_c: after the timestep loop)
    } else {
    // dM[g,c] = A[g,c]^T dX[g] over the non-empty tiles
    {
      GemmArgs a = gg_args();
      a.A = P<u16>(adj, AL.AgT); a.sAp = C * v * AL.vp; a.sAq = v * AL.vp; a.sAm = AL.vp; a.sAk = 1;
      a.B = DXH; a.sBp = v * 2 * H; a.sBk = 2 * H; a.sBn = 1;
      a.D = dM; a.sDz = v * H; a.sDm = H; a.sDn = 1;
      a.zdiv = (int)C; a.Z = (int)(c.b * C); a.zmask = dense_ch ? nullptr : P<unsigned char>(adj, AL.occ);
      a.M = (int)v; a.N = (int)H; a.K = (int)v;
      // dbeta_c += column sums of dM[g,c] (the edge bias enters every message
      // row): per (graph, channel, 32-row slice) partials, summed in a fixed
      // order below (deterministic)
      if (use_bias) { a.csum = dbeta; a.scq = H; a.cpart = P<float>(ws, L.CSP); a.cslots = (int)((v + 31) / 32); }
      if (int e = gg_launch<PREC>(a, true, true, false, K_PROP_BWD, s)) return e;
      if (use_bias) {
        Prof p(K_PROP_BWD, s);
        SumPlan sp(P<float>(ws, L.SUMS));
        const long S = a.cslots;
        SumJob& q = sp.add(a.cpart, (int)c.b, (int)S, C * S * H, H, C * H, H, S * H, dbeta, dbeta, C * H, 1);
        q.ugmax = gmax;
        if (!dense_ch) { q.mask = P<const unsigned char>(adj, AL.occ); q.mT = C; q.mC = 1; }
        if (int e = sp.launch(s)) return e;
      }
    }
    // dh[g] += sum over g's channels of dM[g,c] W_c^T
    {
      GemmArgs a = gg_args();
      a.A = dM; a.sAp = C * v * H; a.sAq = v * H; a.sAm = H; a.sAk = 1;
      a.B = P<float>(pack, PL.gw(c.ed ? t : 0)); a.sBq = H * H; a.sBk = 1; a.sBn = H;
      a.D = DXH + H; a.sDz = v * 2 * H; a.sDm = 2 * H; a.sDn = 1; a.mode = GG_ADD;
      a.tl = P<int>(adj, AL.chl); a.ts = C + 1;
      a.Z = c.b; a.M = (int)v; a.N = (int)H; a.K = (int)H;
      if (int e = gg_launch<PREC>(a, false, true, true, K_PROP_BWD, s)) return e;
    }
    // dW_c (+)= sum over c's graphs of h_t[g]^T dM[g,c]
    {
      float* G_out = c.ed ? P<float>(ws, L.GW) : dW;
      const bool chunked = AL.nch > 1;
      GemmArgs a = gg_args();
      a.A = ht; a.sAq = v * H; a.sAm = 1; a.sAk = H;
      a.B = dM; a.sBp = v * H; a.sBq = C * v * H; a.sBk = H; a.sBn = 1;
      a.D = G_out; a.sDp = H * H; a.sDm = H; a.sDn = 1;
      a.mode = chunked ? GG_ATOMIC : c.ed ? GG_STORE : GG_ADD;
      a.tl = P<int>(adj, AL.cgc); a.ts = AL.gch + 1; a.zdiv = AL.nch;  // z = (channel, chunk of its graphs)
      a.Z = (int)C * AL.nch; a.M = (int)H; a.N = (int)H; a.K = (int)v;
      // chunks of one channel: slab partials, summed in chunk order (added
      // into dW over the timesteps; stored into this timestep's GW under edge dropout)
      if (chunked) { a.slab = P<float>(ws, L.SLAB); a.sSlab = H * H; }
      a.ugmax = gmax;  // final values: / S in the epilogue
      if (int e = gg_launch<WPREC>(a, false, false, false, K_WGRAD, s)) return e;
      Prof p(K_WGRAD, s);
      if (chunked) slab_reduce(a, (int)C, AL.nch, nullptr, 0, c.ed ? 0 : 1, H * H, s);
      if (c.ed)
        hipLaunchKernelGGL(k_gen_wmask_acc, dim3(grid1d(C * ((H + 3) / 4) * H)), dim3(256), 0, s, P<const float>(ws, L.GW), dW,
                           c.C, c.H, t, c.edrop);
    }
    }
    // dL/dh0 (unscaled) after the first timestep; the earlier steps' deltas
    // are formed inside the next k_gen_bwd1
    if (t == 0) {
      Prof p(K_PROP_BWD, s);
      hipLaunchKernelGGL(k_gen_delta, dim3(grid1d((long)c.b * ((c.vin + 3) / 4) * H)), dim3(256), 0, s, DXH, dh0, N,
                         c.H, c.vin, c.sdrop, -1, gmax, 1);
    }
  }
  if (c.sparse) {
    // dW_c = sum_t mask_t (Y_t^T dXg_t), one launch: z = a chunk of <= AL.chunk
    // tiles of one channel (zmap) with every timestep's copy of those tiles as
    // its terms (term q = t * cap_tiles + tile: the slices are cap_tiles tiles
    // apart); under edge dropout the accumulator is masked and banked at each
    // timestep's end (GemmArgs::tgroups), so each chunk adds into dW once per
    // step instead of once per timestep (fp32 atomics: chunks of one channel)
    {
      Prof p(K_WGRAD, s);
      hipLaunchKernelGGL(k_pair_wtl_expand, dim3((unsigned)((AL.zw + 255) / 256)), dim3(256), 0, s,
                         P<const int>(adj, AL.wtl), AL.zw, c.T, AL.cap_tiles, AL.chunk, P<int>(ws, L.WTL));
    }
    GemmArgs a = gg_args();
    a.A = P<float>(ws, L.py(0)); a.sAm = 1; a.sAk = H; a.sAq = PAIR_TILE * H;
    a.B = P<float>(ws, L.pdx(0)); a.sBk = H; a.sBn = 1; a.sBq = PAIR_TILE * H;
    a.D = dW; a.sDp = H * H; a.sDm = H; a.sDn = 1; a.mode = GG_ATOMIC;
    a.tl = P<const int>(ws, L.WTL); a.ts = 1 + (long)c.T * AL.chunk;
    a.zmap = P<const int>(adj, AL.wmap); a.zmask = P<const unsigned char>(adj, AL.wmask);
    a.Z = AL.zw; a.M = (int)H; a.N = (int)H; a.K = PAIR_TILE;
    // a channel's only chunk stores its dW (zmask 2); several chunks: slab
    // partials summed in chunk order (k_slab_reduce, below)
    a.slab = P<float>(ws, L.SLAB); a.sSlab = H * H;
    a.ugmax = gmax;
#ifdef GGNN_TS
    a.tsprobe = 1;
#endif
    // the term-group kernel also without dropout (banks unmasked): it holds
    // two workgroups per CU where the plain ring holds one (round 5: b = 256
    // reference step, dropout off, wgrad 0.96 -> 0.80 ms as the dropout-on run)
    a.tgroups = c.T;
    if (c.ed) {
      a.dr = c.edrop;
      // the masks as bits: written by the pack beside its masked copies
      // (ggnn_pack_weights*, one Philox draw per weight and timestep for both)
      const int w32 = (int)((H + 31) / 32);
      const uint32_t* mb = P<const uint32_t>(pack, PL.gb(0));
      a.mbits = mb; a.mbw = w32; a.mbC = (int)C;
    }
    if (int e = gg_launch<WPREC>(a, false, false, false, K_WGRAD, s)) return e;
    Prof p(K_WGRAD, s);
    slab_reduce(a, (int)C, 0, P<const int>(adj, AL.wst), 1, 0, H * H, s);
  }
  // GRU weight gradients over all T*N rows at once, split-K with fp32
  // atomics, which bound these products at ~65 G adds/s.  Large batches: z =
  // a chunk of rows, its terms the T timesteps' slices of those rows, ~512
  // workgroups (b = 256: 16-30 adds per output instead of 64 with z = (chunk,
  // timestep); wgrad 0.795 -> 0.691 ms per step at the reference
  // configuration).  Small batches (fewer than one 128-row chunk per
  // workgroup slot): z = (chunk, timestep), ~1024 workgroups of short walks,
  // which measured faster there (20 sentences: 0.303 vs 0.336 ms)
  {
    auto wg = [&](size_t aoff, long slotA, size_t boff, long ldB, long slotB, int Nn, float* out, long ldO) {
      const GenWgPlan pl = gen_wg_plan(c, Nn);
      GemmArgs a = gg_args();
      a.A = P<float>(ws, aoff); a.sAq = slotA; a.sAm = 1; a.sAk = H;
      a.B = P<float>(ws, boff); a.sBq = slotB; a.sBk = ldB; a.sBn = 1;
      a.D = out; a.sDm = ldO; a.sDn = 1; a.mode = GG_ATOMIC;
      a.M = (int)H; a.N = Nn; a.Ktot = N;
      a.nterm = pl.nterm; a.zdiv = pl.zdiv; a.Z = pl.Z;
      a.sAp = pl.KC * H; a.sBp = pl.KC * ldB; a.K = (int)pl.KC; a.sKp = pl.KC;
      // the z partials in a slab, summed in z order (deterministic)
      a.slab = P<float>(ws, L.SLAB); a.sSlab = H * Nn;
      a.ugmax = gmax;
#ifdef GGNN_TS
      a.tsprobe = out == dWc ? 2 : 0;
#endif
      if (int e = gg_launch<WPREC>(a, false, false, false, K_WGRAD, s)) return e;
      Prof p(K_WGRAD, s);
      slab_reduce(a, 1, a.Z, nullptr, 0, 0, 0, s);
      return (int)GGNN_OK;
    };
    const long sl = (long)L.nh;  // floats between timestep slots of an [N][H] array
    if (int e = wg(L.x(0), sl, L.dzc(0), H, sl, (int)H, dWc, H)) return e;
    if (int e = wg(L.rh(0), sl, L.dzc(0), H, sl, (int)H, dWc + H * H, H)) return e;
    if (int e = wg(L.x(0), sl, L.dzg(0), 2 * H, 2 * sl, (int)(2 * H), dWg, 2 * H)) return e;
    if (int e = wg(L.hsl(0), sl, L.dzg(0), 2 * H, 2 * sl, (int)(2 * H), dWg + H * 2 * H, 2 * H)) return e;
  }
  {
    Prof p(K_IO, s);
    // bias gradients: fixed-order sums of the per-(timestep, slice) GRU bias
    // rows and of pair mode's per-(timestep, tile) dbeta partials
    SumPlan sp(P<float>(ws, L.SUMS));
    const int nsl = (int)gen_bias_slices(c);
    // (these sums, and every weight-gradient product's epilogue, GemmArgs::ugmax,
    // carry the unscale 1 / S: no separate pass over the gradients)
    if (fuse2) {
      // dbg_r from the fused epilogue's rows, dbg_u | dbc from k_gen_bwd1's
      sp.rows(P<const float>(ws, L.GBR), c.T, gbr_rows, gbr_rows, H, dbg, nullptr, H).ugmax = gmax;
      sp.add(P<const float>(ws, L.GBP) + H, c.T, nsl, (long)nsl * 3 * H, 3 * H, 2 * H, 2 * H, 0, dbg + H, dbc, H)
          .ugmax = gmax;
    } else {
      sp.rows(P<const float>(ws, L.GBP), c.T, nsl, nsl, 3 * H, dbg, dbc, 2 * H).ugmax = gmax;
    }
    if (int e = sp.launch(s)) return e;
    if (c.sparse && use_bias) {
      GemmArgs r = gg_args();
      r.slab = P<float>(ws, L.PDB); r.sSlab = H; r.D = dbeta; r.sDm = 0; r.M = 1; r.N = (int)H;
      slab_reduce_t(r, (int)C, P<const int>(adj, AL.poff), PAIR_TILE, c.T, AL.cap_tiles, s, gmax);
    }
  }
  LAUNCHCHK();
  return GGNN_OK;
}
