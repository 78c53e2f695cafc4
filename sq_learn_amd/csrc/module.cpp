// CPython extension module ``sq_learn_amd._C``: thin argument marshalling to
// the extern "C" launchers of the .hip translation units.  Pointers arrive as
// integers (tensor.data_ptr()), the HIP stream as the integer handle of
// torch.cuda.current_stream(), so every launch is stream-ordered with torch
// and capturable in a hipGraph.  No torch C++ headers: the native layer is
// ABI-independent of the torch build.
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <hip/hip_runtime.h>

extern "C" {
// qrand.hip
__attribute__((weak)) int sq_trunc_normal_add(void*, int, long long, double, unsigned, unsigned, unsigned, unsigned,
                        unsigned long long, void*);
__attribute__((weak)) int sq_philox_normal(void*, int, long long, double, double, unsigned, unsigned, unsigned, unsigned,
                     unsigned long long, void*);
__attribute__((weak)) int sq_philox_uniform(void*, long long, unsigned, unsigned, unsigned, unsigned, unsigned long long,
                      void*);
__attribute__((weak)) int sq_ae_batch(const void*, const void*, void*, long long, int, unsigned, unsigned, unsigned,
                unsigned, unsigned long long, void*);
__attribute__((weak)) int sq_pe_batch(const void*, const void*, void*, long long, unsigned, unsigned, unsigned, unsigned,
                unsigned long long, void*);
// tomography.hip
__attribute__((weak)) int sq_tomography(const void*, int, int, const void*, int, int, const void*,
                                        void*, void*, int, unsigned, unsigned, unsigned, unsigned,
                                        long long, void*, double);
__attribute__((weak)) int sq_mnom_segments(const void*, long long, const void*, long long,
                                           long long, const void*, void*, long long, unsigned,
                                           unsigned, unsigned, unsigned, const void*, int, void*);
__attribute__((weak)) int sq_bounds_filter(const void*, void*, void*, const void*, const void*,
                                           long long, double, void*, void*, const void*, void*,
                                           void*, const void*, const void*, int, int, void*, void*,
                                           void*);
__attribute__((weak)) int sq_multi_records(void*, void*, int, int, int, const void*, const void*,
                                           long long, void*, void*, void*);
__attribute__((weak)) int sq_set_overflow2(void*, void*);
__attribute__((weak)) int sq_shift_operand(const void*, const void*, int, int, int, int, double,
                                           void*, void*, void*, int, int, unsigned, void*);
__attribute__((weak)) int sq_fast_centroids(void*, const void*, const void*, int, int, int, void*,
                                            void*, void*, void*);
// tsgemm64.hip
__attribute__((weak)) int sq_xtx(const void*, int, long long, const void*, int, const void*, int,
                                 long long, const void*, int, long long, int, int, void*, void*,
                                 int, void*);
__attribute__((weak)) int sq_xtx_geometry(int, int, int, int*, int*, int*);
__attribute__((weak)) int sq_xw(const void*, int, long long, const void*, long long, int,
                                const void*, long long, int, int, void*, int, long long, void*);
// ipe.hip
__attribute__((weak)) int sq_ipe_fused(const void*, long long, const void*, const void*,
                                       const void*, const void*, const void*, void*, void*,
                                       long long, int, int, int, int, double, int, unsigned,
                                       unsigned, unsigned, unsigned, unsigned, unsigned, unsigned,
                                       unsigned, unsigned, unsigned, unsigned, unsigned, long long,
                                       int, void*, void*, void*, const void*, const void*,
                                       long long, const void*, const void*);
// ipe16.hip
__attribute__((weak)) int sq_ipe16(int, const long long*, const double*, void*);
// kmpp.hip, batched restarts
__attribute__((weak)) int sq_kmpp_batch(int, const long long*, void*);
__attribute__((weak)) int sq_centroid_delta(const void*, const void*, const void*, void*, void*,
                                            void*, long long, int, int, int, int, void*, void*,
                                            void*, void*);
__attribute__((weak)) int sq_centroid_delta_lists(const void*, const void*, const void*, void*,
                                                  void*, void*, long long, int, int, int, int,
                                                  void*, void*, void*, const void*, const void*,
                                                  const void*, const void*, const void*,
                                                  const void*, void*);
__attribute__((weak)) int sq_cluster_inertia(const void*, const void*, const void*, const void*,
                                             int, int, int, int, void*, void*);
// pairwise_fast.hip
__attribute__((weak)) int sq_pairwise_reduce(const void*, const void*, void*, int, int, int, int,
                                             double, int, void*);
// forest.hip
__attribute__((weak)) int sq_forest_apply(const void*, const void*, const void*, const void*,
                                          const void*, int, const void*, long long, int, void*,
                                          void*);
__attribute__((weak)) int sq_forest_predict(const void*, const void*, const void*, const void*,
                                            const void*, const void*, int, const void*, int,
                                            const void*, long long, int, double, void*, void*);
// elkan.hip
__attribute__((weak)) int sq_elkan_step(const void*, const void*, const void*, const void*,
                                        const void*, void*, void*, void*, long long, int, int,
                                        int, int, void*);
// failure.hip
__attribute__((weak)) int sq_failure_inject(void*, long long, int, double, int, unsigned, unsigned,
                                            unsigned, unsigned, unsigned, unsigned, unsigned,
                                            unsigned, long long, void*, void*, void*, void*,
                                            const void*, long long, const void*, int, int, void*);
// kmeans.hip
__attribute__((weak)) int sq_estep_bf16(const void* X, const void* C, void* inertia_part, const void* cn,
                  const void* xn, void* labels, void* mind, void* ovf_rows, void* ovf_count,
                  void* inertia, long long n, int d, int k, int k_pad, double delta, int part_cap,
                  unsigned k0, unsigned k1, unsigned s0, unsigned s1, long long row_offset,
                  int ovf_cap, void* stream);
__attribute__((weak)) int sq_band_select(const void* D, const void* rows, const void* xn, void* labels, void* mind,
                   long long m, int k, long long ldD, double delta, unsigned k0, unsigned k1,
                   unsigned s0, unsigned s1, long long row_offset, void* stream);
__attribute__((weak)) int sq_band_select_rows(const void*, const void*, const void*, const void*, const void*,
                        const void*, void*, long long, int, int, int, double, unsigned, unsigned,
                        unsigned, unsigned, long long, void*);
__attribute__((weak)) int sq_centroid_accumulate(const void* X, int xdtype, const void* labels, const void* weights,
                           void* sums, void* counts, long long n, int d, int k, int chunk,
                           void* stream);
__attribute__((weak)) int sq_centroid_reduce(const void*, int, const void*, const void*, void*, void*,
                       long long, int, int, int, int, void*, void*, void*, void*, const void*,
                       void*);
__attribute__((weak)) int sq_centroid_finalize(const void* packed, const void* C_old, void* C_new, void* C_bf16,
                         void* C_lo, void* cn, void* shift, int k, int d, int k_pad, double noise_b,
                         unsigned k0, unsigned k1, unsigned s0, unsigned s1, int empty_policy,
                         void* scalars, void* ovf_count, void* C_f16, double alpha, void* cmax2,
                         const void* kept, void* stream);
__attribute__((weak)) int sq_estep_x64(const void*, const void*, const void*, const void*,
                                       const void*, const void*, void*, void*, void*, void*, void*,
                                       void*, void*, void*, void*, void*, void*, void*, void*,
                                       void*, void*, int, long long, int, int, int, int, double,
                                       double, unsigned,
                                       unsigned, unsigned, unsigned, long long, int, void*);
__attribute__((weak)) int sq_fill_mind(const void*, int, const void*, int, const void*, void*,
                                       long long, void*);
__attribute__((weak)) int sq_sum_f32(const void*, long long, void*, int, void*, void*);
// kmpp.hip
__attribute__((weak)) int sq_kmpp_grid(long long);
__attribute__((weak)) int sq_kmpp_init(const void*, long long, int, long long, const void*,
                                       const void*, void*, void*, void*, void*, int, void*, void*,
                                       void*, void*);
__attribute__((weak)) int sq_kmpp_block_totals(const void*, const void*, long long, long long, int,
                                               double, void*, void*);
__attribute__((weak)) int sq_kmpp_cc(const void*, const void*, int, int, int, void*, int, void*,
                                     void*, int, void*, long long, void*, void*);
__attribute__((weak)) int sq_kmpp_screen(void*, void*, const void*, const void*, const void*, int,
                                         const void*, int, int, long long, long long, int, void*,
                                         void*, void*, void*, void*, int, void*);
__attribute__((weak)) int sq_kmpp_dots(const void*, int, long long, const void*, void*, void*);
__attribute__((weak)) int sq_kmpp_bound(const void*, int, const void*, const void*, const void*,
                                        const void*, const void*, const void*, int, int,
                                        long long, long long, int, const void*, const void*,
                                        void*, void*, void*);
__attribute__((weak)) int sq_kmpp_exact(const void*, long long, int, long long, int, const void*,
                                        const void*, const void*, double, const void*,
                                        const void*, void*, void*, void*, long long, int, void*);
__attribute__((weak)) int sq_kmpp_pick(const void*, int, long long, long long, const void*, int,
                                       const void*, const void*, const void*, const void*,
                                       const void*, double, void*, const void*, long long, int,
                                       void*, void*, long long, long long, void*);
__attribute__((weak)) int sq_kmpp_finish(const void*, int, int, void*, void*, const void*, void*,
                                         const void*, const void*, int, void*, void*, int, void*,
                                         void*);
// estep_f32.hip
__attribute__((weak)) int sq_estep_f32(const void*, const void*, const void*, void*, void*, void*,
                                       void*, void*, int, void*, long long, int, int, double,
                                       double, unsigned, unsigned, unsigned, unsigned, long long,
                                       int, void*);
__attribute__((weak)) int sq_rows_f64(const void*, long long, const void*, long long, int, int,
                                      const void*, const void*, long long, long long, void*, void*,
                                      void*, void*, double, unsigned, unsigned, unsigned, unsigned,
                                      long long, int, void*);
__attribute__((weak)) int sq_centers_f16_operand(const void*, void*, int, int, int, int, double,
                                                 void*);
__attribute__((weak)) int sq_mstep_stats(const void*, const void*, const void*, const void*, int, int,
                                         int, int, const void*, long long, void*, void*, void*,
                                         void*);
__attribute__((weak)) int sq_pack_stats(const void* sums, const void* counts, const void* inertia,
                                        void* packed, int k, int d, int xexp, int wexp, void*);
__attribute__((weak)) int sq_ipe_estep(const void* G, const void* xn, const void* cn, void* labels, void* mind,
                 long long m, int k, long long ldG, double eps, int Q, unsigned k0, unsigned k1,
                 unsigned s0, unsigned s1, long long row_offset, void* stream);
// linalg.hip
__attribute__((weak)) int sq_col_moments(const void*, int, long long, long long, int, void*, int,
                                         void*);
__attribute__((weak)) int sq_mu_sums(const void*, int, long long, const void*, int, void*, void*,
                                     void*, int, void*, long long, int, const void*, float, void*);
__attribute__((weak)) int sq_row_norms(const void* X, int xdtype, void* out, long long n, int d, void* stream);
// knn.hip
__attribute__((weak)) int sq_knn_topk(const void* D, void* outd, void* outi, long long m, int nref, long long ldD, int kk,
                long long col_offset, void* stream);
}

#define CHECK(fn) if (!(fn)) { PyErr_SetString(PyExc_RuntimeError, "native symbol " #fn " not built"); return nullptr; }
static PyObject* ret(int rc) {
  if (rc != 0) {
    PyErr_Format(PyExc_RuntimeError, "sq_learn_amd native launch failed: %s (%d)",
                 hipGetErrorString((hipError_t)rc), rc);
    return nullptr;
  }
  Py_RETURN_NONE;
}

#define P(x) ((void*)(uintptr_t)(x))

static PyObject* py_trunc_normal_add(PyObject*, PyObject* a) {
  unsigned long long x, off, st; int dt; long long n; double b; unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KiLdIIIIKK", &x, &dt, &n, &b, &k0, &k1, &s0, &s1, &off, &st)) return nullptr;
  CHECK(sq_trunc_normal_add)
  int rc; Py_BEGIN_ALLOW_THREADS rc = sq_trunc_normal_add(P(x), dt, n, b, k0, k1, s0, s1, off, P(st)); Py_END_ALLOW_THREADS
  return ret(rc);
}

static PyObject* py_philox_normal(PyObject*, PyObject* a) {
  unsigned long long x, off, st; int dt; long long n; double mu, sd; unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KiLddIIIIKK", &x, &dt, &n, &mu, &sd, &k0, &k1, &s0, &s1, &off, &st)) return nullptr;
  CHECK(sq_philox_normal)
  return ret(sq_philox_normal(P(x), dt, n, mu, sd, k0, k1, s0, s1, off, P(st)));
}

static PyObject* py_philox_uniform(PyObject*, PyObject* a) {
  unsigned long long x, off, st; long long n; unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KLIIIIKK", &x, &n, &k0, &k1, &s0, &s1, &off, &st)) return nullptr;
  CHECK(sq_philox_uniform)
  return ret(sq_philox_uniform(P(x), n, k0, k1, s0, s1, off, P(st)));
}

static PyObject* py_ae_batch(PyObject*, PyObject* a) {
  unsigned long long pa, pe, po, off, st; long long n; int Q; unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KKKLiIIIIKK", &pa, &pe, &po, &n, &Q, &k0, &k1, &s0, &s1, &off, &st)) return nullptr;
  CHECK(sq_ae_batch)
  return ret(sq_ae_batch(P(pa), P(pe), P(po), n, Q, k0, k1, s0, s1, off, P(st)));
}

static PyObject* py_pe_batch(PyObject*, PyObject* a) {
  unsigned long long pw, pm, po, off, st; long long n; unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KKKLIIIIKK", &pw, &pm, &po, &n, &k0, &k1, &s0, &s1, &off, &st)) return nullptr;
  CHECK(sq_pe_batch)
  return ret(sq_pe_batch(P(pw), P(pm), P(po), n, k0, k1, s0, s1, off, P(st)));
}

static PyObject* py_estep_bf16(PyObject*, PyObject* a) {
  unsigned long long X, C, part, cn, xn, lab, mind, ovr, ovc, inr, st;
  long long n, roff; int d, k, kpad, pcap, cap; double delta; unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KKKKKKKKKKLiiidiIIIILiK", &X, &C, &part, &cn, &xn, &lab, &mind, &ovr,
                        &ovc, &inr, &n, &d, &k, &kpad, &delta, &pcap, &k0, &k1, &s0, &s1, &roff,
                        &cap, &st))
    return nullptr;
  CHECK(sq_estep_bf16)
  return ret(sq_estep_bf16(P(X), P(C), P(part), P(cn), P(xn), P(lab), P(mind), P(ovr), P(ovc),
                           P(inr), n, d, k, kpad, delta, pcap, k0, k1, s0, s1, roff, cap, P(st)));
}

static PyObject* py_band_select(PyObject*, PyObject* a) {
  unsigned long long D, rows, xn, lab, mind, st; long long m, ld, roff; int k; double delta;
  unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KKKKKLiLdIIIILK", &D, &rows, &xn, &lab, &mind, &m, &k, &ld, &delta,
                        &k0, &k1, &s0, &s1, &roff, &st))
    return nullptr;
  CHECK(sq_band_select)
  return ret(sq_band_select(P(D), P(rows), P(xn), P(lab), P(mind), m, k, ld, delta, k0, k1, s0, s1,
                            roff, P(st)));
}

static PyObject* py_tomography(PyObject*, PyObject* a) {
  unsigned long long V, sched, first, err, out, st; int r, d, T, mode, ninf; long long roff;
  unsigned k0, k1, s0, s1;
  double stop_err = 0.0;
  if (!PyArg_ParseTuple(a, "KiiKiiKKKiIIIILK|d", &V, &r, &d, &sched, &T, &mode, &first, &err, &out,
                        &ninf, &k0, &k1, &s0, &s1, &roff, &st, &stop_err))
    return nullptr;
  CHECK(sq_tomography)
  return ret(sq_tomography(P(V), r, d, P(sched), T, mode, P(first), P(err), P(out), ninf, k0, k1,
                           s0, s1, roff, P(st), stop_err));
}

static PyObject* py_mnom_segments(PyObject*, PyObject* a) {
  unsigned long long W, wrow, Ns, cnt, sid, st; long long ldw, m, B, ldc; int level;
  unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KLKLLKKLIIIIKiK", &W, &ldw, &wrow, &m, &B, &Ns, &cnt, &ldc, &k0, &k1,
                        &s0, &s1, &sid, &level, &st))
    return nullptr;
  CHECK(sq_mnom_segments)
  return ret(sq_mnom_segments(P(W), ldw, P(wrow), m, B, P(Ns), P(cnt), ldc, k0, k1, s0, s1, P(sid),
                              level, P(st)));
}

static PyObject* py_bounds_filter(PyObject*, PyObject* a) {
  unsigned long long lab, ub, lb, sh, sm, rl, rc, mf, mr, mcnt, cc, fi, st, mc = 0, rcn = 0;
  long long n;
  double delta; int nf, k;
  // optional: corrections to zero, the multi-list head counter
  if (!PyArg_ParseTuple(a, "KKKKKLdKKKKKKKiiK|KK", &lab, &ub, &lb, &sh, &sm, &n, &delta, &rl, &rc,
                        &mf, &mr, &mcnt, &cc, &fi, &nf, &k, &st, &mc, &rcn))
    return nullptr;
  CHECK(sq_bounds_filter)
  return ret(sq_bounds_filter(P(lab), P(ub), P(lb), P(sh), P(sm), n, delta, P(rl), P(rc), P(mf),
                              P(mr), P(mcnt), P(cc), P(fi), nf, k, P(st), P(mc), P(rcn)));
}

// the multi-row records of this thread's next certified E-steps (null: off)
static PyObject* py_multi_records(PyObject*, PyObject* a) {
  unsigned long long rec, mf, dsh, dq, mb, cb, nd; int now, lo, ring; long long ds;
  if (!PyArg_ParseTuple(a, "KKiiiKKLKKK", &rec, &mf, &now, &lo, &ring, &dsh, &dq, &ds, &mb, &cb,
                        &nd))
    return nullptr;
  CHECK(sq_multi_records)
  return ret(sq_multi_records(P(rec), P(mf), now, lo, ring, P(dsh), P(dq), ds, P(mb), P(cb),
                              P(nd)));
}

// the second overflow list of the dense-row 3-pass kernel (null: off)
static PyObject* py_set_overflow2(PyObject*, PyObject* a) {
  unsigned long long rows, cnt;
  if (!PyArg_ParseTuple(a, "KK", &rows, &cnt)) return nullptr;
  CHECK(sq_set_overflow2)
  return ret(sq_set_overflow2(P(rows), P(cnt)));
}

// the gap screen's fp16 shift operand of one centroid update
static PyObject* py_shift_operand(PyObject*, PyObject* a) {
  unsigned long long co, cn, snap, dsh, dq, st; int ldc, d, dp, k, ring, snew; double alpha;
  unsigned valid;
  if (!PyArg_ParseTuple(a, "KKiiiidKKKiiIK", &co, &cn, &ldc, &d, &dp, &k, &alpha, &snap, &dsh,
                        &dq, &ring, &snew, &valid, &st))
    return nullptr;
  CHECK(sq_shift_operand)
  return ret(sq_shift_operand(P(co), P(cn), ldc, d, dp, k, alpha, P(snap), P(dsh), P(dq), ring,
                              snew, valid, P(st)));
}

static PyObject* py_fast_centroids(PyObject*, PyObject* a) {
  unsigned long long sh, sq, C, idx, smr, cc, st; int k, d, nf;
  if (!PyArg_ParseTuple(a, "KKKiiiKKKK", &sh, &sq, &C, &k, &d, &nf, &idx, &smr, &cc, &st))
    return nullptr;
  CHECK(sq_fast_centroids)
  return ret(sq_fast_centroids(P(sh), P(sq), P(C), k, d, nf, P(idx), P(smr), P(cc), P(st)));
}

static PyObject* py_centroid_delta(PyObject*, PyObject* a) {
  unsigned long long X, lab, prev, sums, cnts, q, h, c, pm, st; long long n; int d, k, xe, qe;
  if (!PyArg_ParseTuple(a, "KKKKKKLiiiiKKKK", &X, &lab, &prev, &sums, &cnts, &q, &n, &d, &k, &xe,
                        &qe, &h, &c, &pm, &st))
    return nullptr;
  CHECK(sq_centroid_delta)
  return ret(sq_centroid_delta(P(X), P(lab), P(prev), P(sums), P(cnts), P(q), n, d, k, xe, qe,
                               P(h), P(c), P(pm), P(st)));
}

static PyObject* py_centroid_delta_lists(PyObject*, PyObject* a) {
  unsigned long long X, lab, prev, sums, cnts, q, h, c, pm, l0, c0, l1, c1, l2, c2, st;
  long long n; int d, k, xe, qe;
  if (!PyArg_ParseTuple(a, "KKKKKKLiiiiKKKKKKKKKK", &X, &lab, &prev, &sums, &cnts, &q, &n, &d, &k,
                        &xe, &qe, &h, &c, &pm, &l0, &c0, &l1, &c1, &l2, &c2, &st))
    return nullptr;
  CHECK(sq_centroid_delta_lists)
  return ret(sq_centroid_delta_lists(P(X), P(lab), P(prev), P(sums), P(cnts), P(q), n, d, k, xe,
                                     qe, P(h), P(c), P(pm), P(l0), P(c0), P(l1), P(c1), P(l2),
                                     P(c2), P(st)));
}

static PyObject* py_cluster_inertia(PyObject*, PyObject* a) {
  unsigned long long sums, cnts, q, C, part, st; int k, d, xe, qe;
  if (!PyArg_ParseTuple(a, "KKKKiiiiKK", &sums, &cnts, &q, &C, &k, &d, &xe, &qe, &part, &st))
    return nullptr;
  CHECK(sq_cluster_inertia)
  return ret(sq_cluster_inertia(P(sums), P(cnts), P(q), P(C), k, d, xe, qe, P(part), P(st)));
}

static PyObject* py_xtx(PyObject*, PyObject* a) {
  unsigned long long A, mua, B, mub, part, C, st; int ta, da, tb, db, sym, ns, acc;
  long long lda, ldb, n;
  if (!PyArg_ParseTuple(a, "KiLKiKiLKiLiiKKiK", &A, &ta, &lda, &mua, &da, &B, &tb, &ldb, &mub,
                        &db, &n, &sym, &ns, &part, &C, &acc, &st))
    return nullptr;
  CHECK(sq_xtx)
  return ret(sq_xtx(P(A), ta, lda, P(mua), da, P(B), tb, ldb, P(mub), db, n, sym, ns, P(part),
                    P(C), acc, P(st)));
}

static PyObject* py_xtx_geometry(PyObject*, PyObject* a) {
  int da, db, sym, TM, TN, np;
  if (!PyArg_ParseTuple(a, "iii", &da, &db, &sym)) return nullptr;
  CHECK(sq_xtx_geometry)
  sq_xtx_geometry(da, db, sym, &TM, &TN, &np);
  return Py_BuildValue("(iii)", TM, TN, np);
}

static PyObject* py_xw(PyObject*, PyObject* a) {
  unsigned long long A, mu, W, Y, st; int ta, d, l, upper, to; long long lda, n, ldw, ldy;
  if (!PyArg_ParseTuple(a, "KiLKLiKLiiKiLK", &A, &ta, &lda, &mu, &n, &d, &W, &ldw, &l, &upper,
                        &Y, &to, &ldy, &st))
    return nullptr;
  CHECK(sq_xw)
  return ret(sq_xw(P(A), ta, lda, P(mu), n, d, P(W), ldw, l, upper, P(Y), to, ldy, P(st)));
}

static PyObject* py_ipe_fused(PyObject*, PyObject* a) {
  unsigned long long X, Cf, C, hint, xn, cn, lab, mind, stats, scr, st, rl = 0, rc = 0, et = 0,
                                                                       eh = 0;
  long long ldx, n, roff, ln = 0;
  int d, dp, k, kp, Q;
  double eps; unsigned k0, k1, s0, s1, t0, t1, ts0, ts1, q0, q1, qs0, qs1; int prune;
  if (!PyArg_ParseTuple(a, "KLKKKKKKKLiiiidiIIIIIIIIIIIILiKKK|KKLKK", &X, &ldx, &Cf, &C, &hint,
                        &xn, &cn, &lab, &mind, &n, &d, &dp, &k, &kp, &eps, &Q, &k0, &k1, &s0,
                        &s1, &t0, &t1, &ts0, &ts1, &q0, &q1, &qs0, &qs1, &roff, &prune, &stats,
                        &scr, &st, &rl, &rc, &ln, &et, &eh))
    return nullptr;
  CHECK(sq_ipe_fused)
  return ret(sq_ipe_fused(P(X), ldx, P(Cf), P(C), P(hint), P(xn), P(cn), P(lab), P(mind), n, d,
                          dp, k, kp, eps, Q, k0, k1, s0, s1, t0, t1, ts0, ts1, q0, q1, qs0, qs1,
                          roff, prune, P(stats), P(scr), P(st), P(rl), P(rc), ln, P(et), P(eh)));
}

// kmpp_batch: (op, host int64 args pointer, stream)
static PyObject* py_kmpp_batch(PyObject*, PyObject* a) {
  int op;
  unsigned long long ia, st;
  if (!PyArg_ParseTuple(a, "iKK", &op, &ia, &st)) return nullptr;
  CHECK(sq_kmpp_batch)
  return ret(sq_kmpp_batch(op, (const long long*)(uintptr_t)ia, P(st)));
}

// ipe16: (op, host int64 args pointer, host double args pointer, stream)
static PyObject* py_ipe16(PyObject*, PyObject* a) {
  int op; unsigned long long ia, da, st;
  if (!PyArg_ParseTuple(a, "iKKK", &op, &ia, &da, &st)) return nullptr;
  CHECK(sq_ipe16)
  return ret(sq_ipe16(op, (const long long*)(uintptr_t)ia, (const double*)(uintptr_t)da, P(st)));
}

static PyObject* py_pairwise_reduce(PyObject*, PyObject* a) {
  unsigned long long X, Y, out, st; int n, m, d, op, dt; double p;
  if (!PyArg_ParseTuple(a, "KKKiiiidiK", &X, &Y, &out, &n, &m, &d, &op, &p, &dt, &st))
    return nullptr;
  CHECK(sq_pairwise_reduce)
  return ret(sq_pairwise_reduce(P(X), P(Y), P(out), n, m, d, op, p, dt, P(st)));
}

static PyObject* py_forest_apply(PyObject*, PyObject* a) {
  unsigned long long l, r, f, t, o, X, out, st; int T, d; long long n;
  if (!PyArg_ParseTuple(a, "KKKKKiKLiKK", &l, &r, &f, &t, &o, &T, &X, &n, &d, &out, &st))
    return nullptr;
  CHECK(sq_forest_apply)
  return ret(sq_forest_apply(P(l), P(r), P(f), P(t), P(o), T, P(X), n, d, P(out), P(st)));
}

static PyObject* py_forest_predict(PyObject*, PyObject* a) {
  unsigned long long l, r, f, t, ml, o, v, X, out, st; int T, s_act, d; long long n; double sc;
  if (!PyArg_ParseTuple(a, "KKKKKKiKiKLidKK", &l, &r, &f, &t, &ml, &o, &T, &v, &s_act, &X, &n, &d,
                        &sc, &out, &st))
    return nullptr;
  CHECK(sq_forest_predict)
  return ret(sq_forest_predict(P(l), P(r), P(f), P(t), P(ml), P(o), T, P(v), s_act, P(X), n, d,
                               sc, P(out), P(st)));
}

static PyObject* py_elkan_step(PyObject*, PyObject* a) {
  unsigned long long X, C, hcc, sn, sh, lab, up, lo, st; long long n; int d, k, dt, init;
  if (!PyArg_ParseTuple(a, "KKKKKKKKLiiiiK", &X, &C, &hcc, &sn, &sh, &lab, &up, &lo, &n, &d, &k,
                        &dt, &init, &st))
    return nullptr;
  CHECK(sq_elkan_step)
  return ret(sq_elkan_step(P(X), P(C), P(hcc), P(sn), P(sh), P(lab), P(up), P(lo), n, d, k, dt,
                           init, P(st)));
}

static PyObject* py_failure_inject(PyObject*, PyObject* a) {
  unsigned long long lab, cnt, lb, corr, mind, X, C, st; long long n, roff, ldx; int k, R, ldc, d;
  double p;
  unsigned k0, k1, s0, s1, t0, t1, u0, u1;
  if (!PyArg_ParseTuple(a, "KLidiIIIIIIIILKKKKKLKiiK", &lab, &n, &k, &p, &R, &k0, &k1, &s0, &s1,
                        &t0, &t1, &u0, &u1, &roff, &cnt, &lb, &corr, &mind, &X, &ldx, &C, &ldc,
                        &d, &st))
    return nullptr;
  CHECK(sq_failure_inject)
  return ret(sq_failure_inject(P(lab), n, k, p, R, k0, k1, s0, s1, t0, t1, u0, u1, roff, P(cnt),
                               P(lb), P(corr), P(mind), P(X), ldx, P(C), ldc, d, P(st)));
}

static PyObject* py_band_select_rows(PyObject*, PyObject* a) {
  unsigned long long X, C, cn, xn, rows, cnt, lab, st; long long cap, roff; int dp, k, kp;
  double delta; unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KKKKKKKLiiidIIIILK", &X, &C, &cn, &xn, &rows, &cnt, &lab, &cap, &dp,
                        &k, &kp, &delta, &k0, &k1, &s0, &s1, &roff, &st))
    return nullptr;
  CHECK(sq_band_select_rows)
  return ret(sq_band_select_rows(P(X), P(C), P(cn), P(xn), P(rows), P(cnt), P(lab), cap, dp, k, kp,
                                 delta, k0, k1, s0, s1, roff, P(st)));
}

static PyObject* py_centroid_accumulate(PyObject*, PyObject* a) {
  unsigned long long X, lab, w, sums, counts, st; int xdt, d, k, chunk; long long n;
  if (!PyArg_ParseTuple(a, "KiKKKKLiiiK", &X, &xdt, &lab, &w, &sums, &counts, &n, &d, &k, &chunk, &st))
    return nullptr;
  CHECK(sq_centroid_accumulate)
  return ret(sq_centroid_accumulate(P(X), xdt, P(lab), P(w), P(sums), P(counts), n, d, k, chunk, P(st)));
}

static PyObject* py_centroid_reduce(PyObject*, PyObject* a) {
  unsigned long long X, lab, w, sums, counts, h, c, pm, mind, cold, st; int xdt, d, k, xe, we;
  long long n;
  if (!PyArg_ParseTuple(a, "KiKKKKLiiiiKKKKKK", &X, &xdt, &lab, &w, &sums, &counts, &n, &d, &k, &xe,
                        &we, &h, &c, &pm, &mind, &cold, &st))
    return nullptr;
  CHECK(sq_centroid_reduce)
  return ret(sq_centroid_reduce(P(X), xdt, P(lab), P(w), P(sums), P(counts), n, d, k, xe, we, P(h),
                                P(c), P(pm), P(mind), P(cold), P(st)));
}

static PyObject* py_estep_x64(PyObject*, PyObject* a) {
  unsigned long long Xh, X, C, Cm, xn, cm2, lab, mind, dr, ovr, mr, mc, corr, rl, rc, ub, lb, ms,
      xr, cnt, part, st;
  int pcap, d, dp, k, kp, list_rs = 0; long long n, roff; double alpha, delta;
  unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KKKKKKKKKKKKKKKKKKKKKiLiiiiddIIIILK|i", &Xh, &X, &C, &Cm, &xn, &cm2,
                        &lab, &mind, &dr, &ovr, &mr, &mc, &corr, &rl, &rc, &ub, &lb, &ms, &xr, &cnt,
                        &part, &pcap,
                        &n, &d, &dp, &k, &kp, &alpha, &delta, &k0, &k1, &s0, &s1, &roff, &st,
                        &list_rs))
    return nullptr;
  CHECK(sq_estep_x64)
  return ret(sq_estep_x64(P(Xh), P(X), P(C), P(Cm), P(xn), P(cm2), P(lab), P(mind), P(dr), P(ovr),
                          P(mr), P(mc), P(corr), P(rl), P(rc), P(ub), P(lb), P(ms), P(xr), P(cnt),
                          P(part), pcap,
                          n, d, dp, k, kp, alpha, delta, k0, k1, s0, s1, roff, list_rs, P(st)));
}

static PyObject* py_fill_mind(PyObject*, PyObject* a) {
  unsigned long long X, Cm, lab, mind, st; int ldx, d; long long n;
  if (!PyArg_ParseTuple(a, "KiKiKKLK", &X, &ldx, &Cm, &d, &lab, &mind, &n, &st)) return nullptr;
  CHECK(sq_fill_mind)
  return ret(sq_fill_mind(P(X), ldx, P(Cm), d, P(lab), P(mind), n, P(st)));
}

static PyObject* py_kmpp_grid(PyObject*, PyObject* a) {
  long long n;
  if (!PyArg_ParseTuple(a, "L", &n)) return nullptr;
  CHECK(sq_kmpp_grid)
  return PyLong_FromLong(sq_kmpp_grid(n));
}

static PyObject* py_kmpp_init(PyObject*, PyObject* a) {
  unsigned long long X, c0, w, cl, nr, bm, Xq, sr, er, q2, st; long long ldx, n; int d, dq;
  if (!PyArg_ParseTuple(a, "KLiLKKKKKKiKKKK", &X, &ldx, &d, &n, &c0, &w, &cl, &nr, &bm, &Xq, &dq,
                        &sr, &er, &q2, &st))
    return nullptr;
  CHECK(sq_kmpp_init)
  return ret(sq_kmpp_init(P(X), ldx, d, n, P(c0), P(w), P(cl), P(nr), P(bm), P(Xq), dq, P(sr),
                          P(er), P(q2), P(st)));
}

static PyObject* py_kmpp_block_totals(PyObject*, PyObject* a) {
  unsigned long long cl, w, bt, st; long long n, R; int G; double scale;
  if (!PyArg_ParseTuple(a, "KKLLidKK", &cl, &w, &n, &R, &G, &scale, &bt, &st)) return nullptr;
  CHECK(sq_kmpp_block_totals)
  return ret(sq_kmpp_block_totals(P(cl), P(w), n, R, G, scale, P(bt), P(st)));
}

static PyObject* py_kmpp_cc(PyObject*, PyObject* a) {
  unsigned long long cand, C, cc, ci, cq, dp, cnt, st; int c, d, t, ldcc, dq; long long ndp;
  if (!PyArg_ParseTuple(a, "KKiiiKiKKiKLKK", &cand, &C, &c, &d, &t, &cc, &ldcc, &ci, &cq, &dq, &dp,
                        &ndp, &cnt, &st))
    return nullptr;
  CHECK(sq_kmpp_cc)
  return ret(sq_kmpp_cc(P(cand), P(C), c, d, t, P(cc), ldcc, P(ci), P(cq), dq, P(dp), ndp, P(cnt),
                        P(st)));
}

static PyObject* py_kmpp_screen(PyObject*, PyObject* a) {
  unsigned long long cl, nr, mp, Dp, bp, cc, mo, sv, ex, sc, ec, st; int cp, ldcc, t, G, prune;
  long long n, R;
  if (!PyArg_ParseTuple(a, "KKKKKiKiiLLiKKKKKiK", &cl, &nr, &mp, &Dp, &bp, &cp, &cc, &ldcc, &t, &n,
                        &R, &G, &mo, &sv, &ex, &sc, &ec, &prune, &st))
    return nullptr;
  CHECK(sq_kmpp_screen)
  return ret(sq_kmpp_screen(P(cl), P(nr), P(mp), P(Dp), P(bp), cp, P(cc), ldcc, t, n, R, G, P(mo),
                            P(sv), P(ex), P(sc), P(ec), prune, P(st)));
}

static PyObject* py_kmpp_bound(PyObject*, PyObject* a) {
  unsigned long long Xq, sr, er, q2, cl, cq, ci, sv, sc, ex, ec, st; int dq, t, d, G;
  long long n, R;
  if (!PyArg_ParseTuple(a, "KiKKKKKKiiLLiKKKKK", &Xq, &dq, &sr, &er, &q2, &cl, &cq, &ci, &t, &d, &n,
                        &R, &G, &sv, &sc, &ex, &ec, &st))
    return nullptr;
  CHECK(sq_kmpp_bound)
  return ret(sq_kmpp_bound(P(Xq), dq, P(sr), P(er), P(q2), P(cl), P(cq), P(ci), t, d, n, R, G,
                           P(sv), P(sc), P(ex), P(ec), P(st)));
}

static PyObject* py_kmpp_exact(PyObject*, PyObject* a) {
  unsigned long long X, cand, cl, w, ex, ec, mo, Do, dp, st; long long ldx, n, R; int d, t, G;
  double scale;
  if (!PyArg_ParseTuple(a, "KLiLiKKKdKKKKKLiK", &X, &ldx, &d, &n, &t, &cand, &cl, &w, &scale, &ex,
                        &ec, &mo, &Do, &dp, &R, &G, &st))
    return nullptr;
  CHECK(sq_kmpp_exact)
  return ret(sq_kmpp_exact(P(X), ldx, d, n, t, P(cand), P(cl), P(w), scale, P(ex), P(ec), P(mo),
                           P(Do), P(dp), R, G, P(st)));
}

static PyObject* py_kmpp_dots(PyObject*, PyObject* a) {
  unsigned long long Xq, cq, out, st; int dq; long long n;
  if (!PyArg_ParseTuple(a, "KiLKKK", &Xq, &dq, &n, &cq, &out, &st)) return nullptr;
  CHECK(sq_kmpp_dots)
  return ret(sq_kmpp_dots(P(Xq), dq, n, P(cq), P(out), P(st)));
}

static PyObject* py_kmpp_pick(PyObject*, PyObject* a) {
  unsigned long long bt, v, cl, m, D, b, w, pos, X, cd, ci, st; int G, t, d;
  long long R, n, ldx, roff, ng; double scale;
  if (!PyArg_ParseTuple(a, "KiLLKiKKKKKdKKLiKKLLK", &bt, &G, &R, &n, &v, &t, &cl, &m, &D, &b, &w,
                        &scale, &pos, &X, &ldx, &d, &cd, &ci, &roff, &ng, &st))
    return nullptr;
  CHECK(sq_kmpp_pick)
  return ret(sq_kmpp_pick(P(bt), G, R, n, P(v), t, P(cl), P(m), P(D), P(b), P(w), scale, P(pos),
                          P(X), ldx, d, P(cd), P(ci), roff, ng, P(st)));
}

static PyObject* py_kmpp_finish(PyObject*, PyObject* a) {
  unsigned long long dp, bt, Pp, dn, v, cd, ci, C, ids, bo, st; int G, t, d, c;
  if (!PyArg_ParseTuple(a, "KiiKKKKKKiKKiKK", &dp, &G, &t, &bt, &Pp, &dn, &v, &cd, &ci, &d, &C,
                        &ids, &c, &bo, &st))
    return nullptr;
  CHECK(sq_kmpp_finish)
  return ret(sq_kmpp_finish(P(dp), G, t, P(bt), P(Pp), P(dn), P(v), P(cd), P(ci), d, P(C), P(ids),
                            c, P(bo), P(st)));
}

static PyObject* py_sum_f32(PyObject*, PyObject* a) {
  unsigned long long v, part, out, st; long long n; int extra;
  if (!PyArg_ParseTuple(a, "KLKiKK", &v, &n, &part, &extra, &out, &st)) return nullptr;
  CHECK(sq_sum_f32)
  return ret(sq_sum_f32(P(v), n, P(part), extra, P(out), P(st)));
}

static PyObject* py_mstep_stats(PyObject*, PyObject* a) {
  unsigned long long sums, counts, qsum, C, corr, part, inr, packed, st; int k, d, xe, qe;
  long long n;
  if (!PyArg_ParseTuple(a, "KKKKiiiiKLKKKK", &sums, &counts, &qsum, &C, &k, &d, &xe, &qe, &corr,
                        &n, &part, &inr, &packed, &st))
    return nullptr;
  CHECK(sq_mstep_stats)
  return ret(sq_mstep_stats(P(sums), P(counts), P(qsum), P(C), k, d, xe, qe, P(corr), n, P(part),
                            P(inr), P(packed), P(st)));
}

static PyObject* py_centroid_finalize(PyObject*, PyObject* a) {
  unsigned long long pk, co, cnw, cb, clo, cn, sh, sc, oc, cf, cm2, kp, st; int k, d, kpad, pol;
  double nb, alpha; unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KKKKKKKiiidIIIIiKKKdKKK", &pk, &co, &cnw, &cb, &clo, &cn, &sh, &k, &d,
                        &kpad, &nb, &k0, &k1, &s0, &s1, &pol, &sc, &oc, &cf, &alpha, &cm2, &kp,
                        &st))
    return nullptr;
  CHECK(sq_centroid_finalize)
  return ret(sq_centroid_finalize(P(pk), P(co), P(cnw), P(cb), P(clo), P(cn), P(sh), k, d, kpad, nb,
                                  k0, k1, s0, s1, pol, P(sc), P(oc), P(cf), alpha, P(cm2), P(kp),
                                  P(st)));
}

static PyObject* py_estep_f32(PyObject*, PyObject* a) {
  unsigned long long X, C, xn, lab, mind, ovr, ovc, part, inr, st; int pcap, dp, kp, cap;
  long long n, roff; double alpha, delta; unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KKKKKKKKiKLiiddIIIILiK", &X, &C, &xn, &lab, &mind, &ovr, &ovc, &part,
                        &pcap, &inr, &n, &dp, &kp, &alpha, &delta, &k0, &k1, &s0, &s1, &roff, &cap,
                        &st))
    return nullptr;
  CHECK(sq_estep_f32)
  return ret(sq_estep_f32(P(X), P(C), P(xn), P(lab), P(mind), P(ovr), P(ovc), P(part), pcap, P(inr),
                          n, dp, kp, alpha, delta, k0, k1, s0, s1, roff, cap, P(st)));
}

static PyObject* py_rows_f64(PyObject*, PyObject* a) {
  unsigned long long X, C, rows, cnt, lab, mind, corr, ub, st; long long ldx, ldc, nd, cap, roff;
  int d, k, grid; double delta; unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KLKLiiKKLLKKKKdIIIILiK", &X, &ldx, &C, &ldc, &d, &k, &rows, &cnt, &nd,
                        &cap, &lab, &mind, &corr, &ub, &delta, &k0, &k1, &s0, &s1, &roff, &grid,
                        &st))
    return nullptr;
  CHECK(sq_rows_f64)
  return ret(sq_rows_f64(P(X), ldx, P(C), ldc, d, k, P(rows), P(cnt), nd, cap, P(lab), P(mind),
                         P(corr), P(ub), delta, k0, k1, s0, s1, roff, grid, P(st)));
}

static PyObject* py_centers_f16_operand(PyObject*, PyObject* a) {
  unsigned long long Cm, op, st; int k, d, dp, kp; double alpha;
  if (!PyArg_ParseTuple(a, "KKiiiidK", &Cm, &op, &k, &d, &dp, &kp, &alpha, &st)) return nullptr;
  CHECK(sq_centers_f16_operand)
  return ret(sq_centers_f16_operand(P(Cm), P(op), k, d, dp, kp, alpha, P(st)));
}

static PyObject* py_pack_stats(PyObject*, PyObject* a) {
  unsigned long long s, c, i, p, st; int k, d, xe, we;
  if (!PyArg_ParseTuple(a, "KKKKiiiiK", &s, &c, &i, &p, &k, &d, &xe, &we, &st)) return nullptr;
  CHECK(sq_pack_stats)
  return ret(sq_pack_stats(P(s), P(c), P(i), P(p), k, d, xe, we, P(st)));
}

static PyObject* py_ipe_estep(PyObject*, PyObject* a) {
  unsigned long long G, xn, cn, lab, mind, st; long long m, ld, roff; int k, Q; double eps;
  unsigned k0, k1, s0, s1;
  if (!PyArg_ParseTuple(a, "KKKKKLiLdiIIIILK", &G, &xn, &cn, &lab, &mind, &m, &k, &ld, &eps, &Q,
                        &k0, &k1, &s0, &s1, &roff, &st))
    return nullptr;
  CHECK(sq_ipe_estep)
  return ret(sq_ipe_estep(P(G), P(xn), P(cn), P(lab), P(mind), m, k, ld, eps, Q, k0, k1, s0, s1,
                          roff, P(st)));
}

static PyObject* py_col_moments(PyObject*, PyObject* a) {
  unsigned long long X, part, st; int xdt, d, pw; long long ldx, n;
  if (!PyArg_ParseTuple(a, "KiLLiKiK", &X, &xdt, &ldx, &n, &d, &part, &pw, &st)) return nullptr;
  CHECK(sq_col_moments)
  return ret(sq_col_moments(P(X), xdt, ldx, n, d, P(part), pw, P(st)));
}

static PyObject* py_mu_sums(PyObject*, PyObject* a) {
  unsigned long long X, qs, rm, cs, part, racc, mean, st; int xdt, nq, pw, d; long long n, ldx;
  float qstep;
  if (!PyArg_ParseTuple(a, "KiLKiKKKiKLiKfK", &X, &xdt, &ldx, &qs, &nq, &rm, &cs, &part, &pw,
                        &racc, &n, &d, &mean, &qstep, &st))
    return nullptr;
  CHECK(sq_mu_sums)
  return ret(sq_mu_sums(P(X), xdt, ldx, P(qs), nq, P(rm), P(cs), P(part), pw, P(racc), n, d,
                        P(mean), qstep, P(st)));
}

static PyObject* py_row_norms(PyObject*, PyObject* a) {
  unsigned long long X, out, st; int xdt, d; long long n;
  if (!PyArg_ParseTuple(a, "KiKLiK", &X, &xdt, &out, &n, &d, &st)) return nullptr;
  CHECK(sq_row_norms)
  return ret(sq_row_norms(P(X), xdt, P(out), n, d, P(st)));
}

static PyObject* py_knn_topk(PyObject*, PyObject* a) {
  unsigned long long D, od, oi, st; long long m, ld, coff; int nref, kk;
  if (!PyArg_ParseTuple(a, "KKKLiLiLK", &D, &od, &oi, &m, &nref, &ld, &kk, &coff, &st)) return nullptr;
  CHECK(sq_knn_topk)
  return ret(sq_knn_topk(P(D), P(od), P(oi), m, nref, ld, kk, coff, P(st)));
}

static PyObject* py_device_arch(PyObject*, PyObject*) {
  hipDeviceProp_t prop;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
    Py_RETURN_NONE;
  return Py_BuildValue("(siii)", prop.gcnArchName, prop.multiProcessorCount,
                       (int)prop.maxSharedMemoryPerMultiProcessor, prop.warpSize);
}

static PyMethodDef methods[] = {
    {"forest_apply", py_forest_apply, METH_VARARGS, "leaf ids of (row, tree) pairs"},
    {"forest_predict", py_forest_predict, METH_VARARGS, "sum of leaf values over trees"},
    {"trunc_normal_add", py_trunc_normal_add, METH_VARARGS, "x += TN(-b,b) (Philox keyed)"},
    {"philox_normal", py_philox_normal, METH_VARARGS, "fill with mean+std*N(0,1)"},
    {"philox_uniform", py_philox_uniform, METH_VARARGS, "fill with U(0,1)"},
    {"ae_batch", py_ae_batch, METH_VARARGS, "batched median-of-Q amplitude estimation"},
    {"pe_batch", py_pe_batch, METH_VARARGS, "batched phase estimation"},
    {"estep_bf16", py_estep_bf16, METH_VARARGS, "fused MFMA distance + delta-band E-step"},
    {"band_select", py_band_select, METH_VARARGS, "delta-band selection over distance rows"},
    {"band_select_rows", py_band_select_rows, METH_VARARGS, "device-driven overflow fallback"},
    {"pairwise_reduce", py_pairwise_reduce, METH_VARARGS, "L1 / chi2 / chebyshev / minkowski tiles"},
    {"elkan_step", py_elkan_step, METH_VARARGS, "Elkan bounded k-means assignment"},
    {"failure_inject", py_failure_inject, METH_VARARGS, "Bernoulli estimation failure + resampling"},
    {"tomography", py_tomography, METH_VARARGS, "batched shot-based vector tomography"},
    {"mnom_segments", py_mnom_segments, METH_VARARGS, "segmented multinomial (long vectors)"},
    {"xtx", py_xtx, METH_VARARGS, "fp64 MFMA (A-mu_a)^T (B-mu_b), split-K + fixed-order finalize"},
    {"xtx_geometry", py_xtx_geometry, METH_VARARGS, "xtx tile sizes and pair count"},
    {"xw", py_xw, METH_VARARGS, "fp64 MFMA (A-mu) W"},
    {"bounds_filter", py_bounds_filter, METH_VARARGS, "Hamerly pruning -> active row list"},
    {"multi_records", py_multi_records, METH_VARARGS, "gap records of the multi rows (gap screen)"},
    {"shift_operand", py_shift_operand, METH_VARARGS, "fp16 centroid-shift operand (gap screen)"},
    {"set_overflow2", py_set_overflow2, METH_VARARGS, "second overflow list of the 3-pass kernel"},
    {"fast_centroids", py_fast_centroids, METH_VARARGS, "fastest centroids + Elkan distances"},
    {"centroid_delta", py_centroid_delta, METH_VARARGS, "incremental fixed-point cluster stats"},
    {"centroid_delta_lists", py_centroid_delta_lists, METH_VARARGS,
     "incremental cluster stats over a filtered E-step's row lists"},
    {"cluster_inertia", py_cluster_inertia, METH_VARARGS, "per-cluster inertia from the stats"},
    {"ipe_fused", py_ipe_fused, METH_VARARGS, "fused fp32-MFMA + amplitude-estimation IPE E-step"},
    {"ipe16", py_ipe16, METH_VARARGS, "certified fp16 screen of the IPE E-step (op per phase)"},
    {"kmpp_batch", py_kmpp_batch, METH_VARARGS, "batched k-means++ restarts (op per phase)"},
    {"centroid_accumulate", py_centroid_accumulate, METH_VARARGS, "label-segmented row sums"},
    {"centroid_reduce", py_centroid_reduce, METH_VARARGS, "counting-sort segmented row sums"},
    {"centroid_finalize", py_centroid_finalize, METH_VARARGS, "centroid average + noise + shift"},
    {"mstep_stats", py_mstep_stats, METH_VARARGS, "incremental M-step inertia + packed bucket"},
    {"estep_f32", py_estep_f32, METH_VARARGS, "fp32-faithful fused E-step (fp16 hi/lo MFMA)"},
    {"estep_x64", py_estep_x64, METH_VARARGS, "certified filter E-step + fp64 re-check"},
    {"fill_mind", py_fill_mind, METH_VARARGS, "exact distance to the label for marked rows"},
    {"sum_f32", py_sum_f32, METH_VARARGS, "deterministic sum of a float vector"},
    {"kmpp_grid", py_kmpp_grid, METH_VARARGS, "k-means++ trial pass grid size"},
    {"kmpp_init", py_kmpp_init, METH_VARARGS, "k-means++ first centre distances"},
    {"kmpp_block_totals", py_kmpp_block_totals, METH_VARARGS, "k-means++ fixed-point block totals"},
    {"kmpp_cc", py_kmpp_cc, METH_VARARGS, "k-means++ candidate-centre distances"},
    {"kmpp_screen", py_kmpp_screen, METH_VARARGS, "k-means++ triangle screen + lazy update"},
    {"kmpp_bound", py_kmpp_bound, METH_VARARGS, "k-means++ certified int8 bound"},
    {"kmpp_exact", py_kmpp_exact, METH_VARARGS, "k-means++ exact fp32 trial distances"},
    {"kmpp_dots", py_kmpp_dots, METH_VARARGS, "int8 MFMA dots of the k-means++ bound (test hook)"},
    {"kmpp_finish", py_kmpp_finish, METH_VARARGS, "k-means++ winner of one centre (one rank)"},
    {"kmpp_pick", py_kmpp_pick, METH_VARARGS, "k-means++ two-level potential sampling"},
    {"rows_f64", py_rows_f64, METH_VARARGS, "exact fp64 E-step over a row list (fp64 MFMA)"},
    {"centers_f16_operand", py_centers_f16_operand, METH_VARARGS, "fp16-split centroid operand"},
    {"pack_stats", py_pack_stats, METH_VARARGS, "pack M-step statistics into one fp64 bucket"},
    {"ipe_estep", py_ipe_estep, METH_VARARGS, "IPE-noised distance argmin"},
    {"col_moments", py_col_moments, METH_VARARGS, "fp64 column sums and sums of squares"},
    {"mu_sums", py_mu_sums, METH_VARARGS, "mu(A) power sums for a p-grid"},
    {"row_norms", py_row_norms, METH_VARARGS, "squared row norms"},
    {"knn_topk", py_knn_topk, METH_VARARGS, "per-row k smallest"},
    {"device_arch", py_device_arch, METH_NOARGS, "(arch, CUs, LDS/CU, wave size)"},
    {nullptr, nullptr, 0, nullptr}};

static struct PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_C",
                                    "sq_learn_amd native HIP kernels (gfx950)", -1, methods};

PyMODINIT_FUNC PyInit__C(void) { return PyModule_Create(&moddef); }
