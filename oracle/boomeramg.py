"""Classical AMG as BoomerAMG is configured by the reference (TEST INFRASTRUCTURE ONLY,
see oracle/__init__.py).

``-X_pc_type hypre -X_pc_hypre_type boomeramg`` with the reference's
``petsc-options-inexact:16-24`` (and the f_ / p_ / diff_ / fp_fieldsplit_0_
blocks, :32-40, :48-56, :63-71, :92-100): ``coarsen_type HMIS``,
``interp_type ext+i``, ``P_max 4``, ``agg_nl 1``, ``agg_num_paths 2``,
``grid_sweeps_all 1``, ``no_CF``.  hypre itself is absent from this image and
from the reference tree: this module restates the published
algorithms those options select (Ruge & Stueben 1987; De Sterck, Yang & Heys
2006 -- HMIS; De Sterck, Falgout, Nolting & Yang 2008 -- extended+i; Stueben
2001, App. A -- aggressive coarsening and multipass interpolation) with
PETSc's PCHYPRE defaults for everything the options leave open.  It is the
exact specification libpls's device AMG follows (csrc/boomeramg.cpp builds the
same hierarchy bit for bit: every sum below runs in the order written, no
contraction) and the oracle its GPU tests compare with.  Parity against hypre
is unpinned.

Setup, level l (A_l square CSR, sorted columns), single rank:
* strength (hypre CreateS, theta = strong_threshold 0.25, mu = max_row_sum
  0.9): row i with diagonal d and off-diagonal entries a_ij; no off-diagonals,
  or mu < 1 and |sum_j a_ij| > mu |d| (row sum incl. d, storage order): no
  strong dependencies; else d >= 0: s = min_j a_ij, j strong iff a_ij < theta s;
  d < 0: s = max_j a_ij, j strong iff a_ij > theta s.  S_i = strong j
  (ascending), S^T its transpose (influences).
* HMIS on one rank = the Ruge-Stueben first pass (hypre's HMIS runs RS pass 1
  inside each process, then PMIS only across process boundaries):
  lambda_i = |S^T_i|; points with S_i empty and lambda_i = 0 are F; then in
  ascending order every undecided point with lambda_i = 0 becomes F; then
  repeatedly the undecided point of largest lambda (ties: smallest index)
  becomes C, its undecided influencees j in S^T_i become F, and a point j that
  becomes F raises lambda_k by 1 for its undecided dependencies k in S_j (in
  order); the undecided dependencies k in S_i of the new C point lose 1, and
  one reaching 0 becomes F.  Left-over undecided points are F.
* aggressive coarsening on the first agg_nl levels (agg_num_paths p): HMIS on
  S gives C1; S2 on C1: j in C1 (j != i) is a strong dependency of i in C1
  iff [j in S_i] + #{k in S_i : j in S_k} >= p; HMIS on S2 (C1's points in
  ascending order) gives C.
* interpolation: C points inject (P_i = e_c(i), coarse points numbered in
  ascending order).  Aggressive levels: multipass (Stueben A.4.3): pass 0 = C;
  pass p = the undecided F points with a strong dependency assigned in an
  earlier pass (decided from the passes before p); Q_i = those
  dependencies (ascending); with a^- = min(a, 0), a^+ = max(a, 0) summed over
  the row's off-diagonals (storage order) and over Q_i: a negative (positive)
  Q-sum of 0 adds the row's negative (positive) sum to d~ = a_ii, else
  alpha = row sum / Q sum for that sign; P_i = sum_{k in Q_i} (-alpha_sign(a_ik)
  a_ik / d~) P_k (Q order, then P_k's storage order); points never reached
  interpolate nothing.  Other levels: extended+i: C^_i = strong C neighbours
  plus the strong C neighbours of strong F neighbours; w_j starts at a_ij for
  j in C^_i (row storage order; weak neighbours in C^_i included) and d~ = a_ii
  plus every other weak a_in; each strong F neighbour k (ascending) spreads
  a_ik over bar(a_kl) = a_kl if a_kl a_kk < 0 else 0: D = sum over k's row
  (storage order) of bar(a_kl) for l in C^_i or l = i; D = 0 adds a_ik to
  d~, else with hypre's distribute = a_ik / D: w_l += distribute bar(a_kl) for
  l in C^_i and d~ += distribute bar(a_ki);
  P_ij = -w_j / d~.  Then P_max truncation: rows with more than P_max entries
  keep the P_max largest |P_ij| (ties: smaller j), rescaled by (row sum) /
  (kept sum) (both in column order) when the kept sum is nonzero.  Exact
  zeros are dropped.
* R = P^T, A_{l+1} = R (A P) (scipy's csr_matmat order);
* levels stop when n <= 9 (hypre's max_coarse_size) or max_levels (25) is
  reached, or when coarsening selects no or every point; the coarsest level is
  solved exactly (hypre's relax type 9, Gaussian elimination).
V-cycle (one PC application, x = 0): per level, grid_sweeps_all sweeps of
hybrid symmetric Gauss-Seidel (PETSc's PCHYPRE default relax type, hypre 6),
lexicographic with no_CF, else over the C points then the F points going
down and F then C going up (hypre's CF relaxation order); r = b - A x;
recurse on R r from 0; x += P e; post-smooth.
* hybrid symmetric Gauss-Seidel with K chunks (libpls option
  ``pls.hypre_relax_chunks``, default 256 -- hypre's relax type 6 as its
  OpenMP build runs it with K threads, par_relax.c): the level's n rows are
  cut into K_l = min(K, n // R, n) contiguous chunks, at least 1, with R =
  ``pls.hypre_relax_min_rows`` (default 1024; 0: no floor) -- undamped
  hybrid sweeps over chunks of ~100 rows diverge on the undrained footing
  solid block (footing N=12: 500 its at K_l = 64, 50 at one chunk, 53 with
  R = 1024, measured with this oracle) -- (size n / K_l, the first n % K_l
  chunks one row longer); u_old = u at the start of the sweep; within chunk c,
  row by row forward and then backward over the chunk's points of the set,
  u_i = (b_i - sum_{j != i} a_ij v_j) / a_ii with v_j = u_j for j in c and
  v_j = u_old_j otherwise (``hybrid_sgs_literal`` is that loop).  In matrix
  form, with A_c the chunk-block-diagonal part of A restricted to the set I
  (D its diagonal, L / U its strict triangles): u_I += M^-1 (b - A u_old)_I,
  M = (D + L) D^-1 (D + U) -- forward d1 = (D + L)^-1 r, the backward sweep's
  right-hand side is r - A_c d1 = -U d1, d2 = (D + U)^-1 (-U d1), and
  d1 + d2 = (D + U)^-1 D d1.  K = 1 is plain symmetric Gauss-Seidel.
"""
from __future__ import annotations

import heapq

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from .options import get as opt

_SUPPORTED_COARSEN = ("HMIS",)
_SUPPORTED_INTERP = ("ext+i",)


def _rows(A):
    A = A.tocsr()
    A.sort_indices()
    return A, A.indptr, A.indices, A.data


def strength(A, theta=0.25, max_row_sum=0.9):
    """S as a list of int arrays (strong dependencies of each row, ascending)."""
    A, rp, ci, v = _rows(A)
    n = A.shape[0]
    S = []
    for i in range(n):
        cols, vals = ci[rp[i]:rp[i + 1]], v[rp[i]:rp[i + 1]]
        d = 0.0
        rs = 0.0
        off = []
        for j, a in zip(cols.tolist(), vals.tolist()):
            rs += a
            if j == i:
                d = a
            else:
                off.append((j, a))
        if not off or (max_row_sum < 1.0 and abs(rs) > max_row_sum * abs(d)):
            S.append(np.zeros(0, dtype=np.int64))
            continue
        if d >= 0.0:
            s = min(a for _, a in off)
            st = [j for j, a in off if a < theta * s]
        else:
            s = max(a for _, a in off)
            st = [j for j, a in off if a > theta * s]
        S.append(np.asarray(st, dtype=np.int64))
    return S


def transpose_lists(S, n):
    T = [[] for _ in range(n)]
    for i, row in enumerate(S):
        for j in row.tolist():
            T[j].append(i)
    return [np.asarray(t, dtype=np.int64) for t in T]


U, F, C = 0, -1, 1


def rs_first_pass(S, n):
    """C/F marker (1 / -1) of the Ruge-Stueben first pass (HMIS on one rank)."""
    ST = transpose_lists(S, n)
    lam = [len(t) for t in ST]
    state = [U] * n
    heap = []

    def make_f(j):
        state[j] = F
        for k in S[j].tolist():
            if state[k] == U:
                lam[k] += 1
                heapq.heappush(heap, (-lam[k], k))

    for i in range(n):
        if len(S[i]) == 0 and lam[i] == 0:
            state[i] = F
    for i in range(n):
        if state[i] == U and lam[i] == 0:
            make_f(i)
    for i in range(n):
        if state[i] == U:
            heapq.heappush(heap, (-lam[i], i))
    while heap:
        nl, i = heapq.heappop(heap)
        if state[i] != U or -nl != lam[i]:
            continue
        state[i] = C
        for j in ST[i].tolist():
            if state[j] == U:
                make_f(j)
        for k in S[i].tolist():
            if state[k] == U:
                lam[k] -= 1
                if lam[k] == 0:
                    make_f(k)
                else:
                    heapq.heappush(heap, (-lam[k], k))
    return np.asarray([C if s == C else F for s in state], dtype=np.int64)


def second_strength(S, cf, num_paths):
    """S2 over the C points (local numbering, ascending original index)."""
    cpts = np.flatnonzero(cf == C)
    loc = -np.ones(len(cf), dtype=np.int64)
    loc[cpts] = np.arange(len(cpts))
    S2 = []
    for i in cpts.tolist():
        cnt = {}
        for k in S[i].tolist():
            if loc[k] >= 0 and k != i:
                cnt[k] = cnt.get(k, 0) + 1
        for k in S[i].tolist():
            for j in S[k].tolist():
                if loc[j] >= 0 and j != i:
                    cnt[j] = cnt.get(j, 0) + 1
        S2.append(np.asarray(sorted(loc[j] for j, c in cnt.items() if c >= num_paths), dtype=np.int64))
    return S2, cpts


def rs_partitioned(S, n, part):
    """The Ruge-Stueben first pass run independently inside every partition
    (part[i]: the partition of point i, contiguous ranges) on the strong
    connections inside it -- HMIS's per-process first pass."""
    if part is None or n == 0 or part[-1] == part[0]:
        return rs_first_pass(S, n)
    cf = np.empty(n, dtype=np.int64)
    starts = np.flatnonzero(np.r_[True, part[1:] != part[:-1]])
    ends = np.r_[starts[1:], n]
    for a, b in zip(starts.tolist(), ends.tolist()):
        Sl = [row[(row >= a) & (row < b)] - a for row in S[a:b]]
        cf[a:b] = rs_first_pass(Sl, b - a)
    return cf


def coarsen_partition(S, n, K, max_cut=0.02):
    """Automatic HMIS partition: the most partitions (<= K, halving) whose
    boundaries cut at most max_cut of the strong connections (a partition
    narrower than the matrix's coupling range would coarsen the boundary
    layers independently); None when even two partitions cut more."""
    if n == 0:
        return None
    rows = np.repeat(np.arange(n), [len(r) for r in S])
    cols = np.concatenate(S) if len(S) else np.zeros(0, dtype=np.int64)
    while K > 1:
        part = chunk_ids(n, K)
        if cols.size == 0 or np.count_nonzero(part[rows] != part[cols]) <= max_cut * cols.size:
            return part
        K //= 2
    return None


def hypre_rand(seed, count):
    """``count`` values of hypre_Rand() after hypre_SeedRand(seed) (hypre's
    utilities/random.c: the Park-Miller minimal standard generator, a = 16807,
    m = 2^31 - 1 by Schrage's method, q = 127773, r = 2836; value = seed / m)."""
    out = np.empty(count, dtype=np.float64)
    s = int(seed)
    for k in range(count):
        hi, lo = divmod(s, 127773)
        t = 16807 * lo - 2836 * hi
        s = t if t > 0 else t + 2147483647
        out[k] = s / 2147483647.0
    return out


def _pattern(S, n):
    lens = np.asarray([len(r) for r in S], dtype=np.int64)
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    cols = np.concatenate(S).astype(np.int64) if len(S) and lens.sum() else np.zeros(0, dtype=np.int64)
    return rows, cols


def pmis_stage(S, n, cf, part=None):
    """HMIS's second stage (De Sterck, Yang & Heys 2006; hypre's CoarsenHMIS =
    the Ruge-Stueben first pass inside every process, then CoarsenPMIS with
    the first pass as the initial splitting, CF_init = 1):
    * measure_i = |S^T_i| + a random number in [0, 1): process (partition) k
      draws hypre_Rand() for its rows in order after hypre_SeedRand(2747 + k)
      (hypre_BoomerAMGIndepSetInit);
    * points without a strong dependency on another partition's point keep
      their first-pass decision; the boundary points (a strong dependency on
      another partition's point: hypre's S_offd) are undecided, or F when
      |S^T_i| = 0 (measure < 1: no point depends on it) -- one partition
      (np = 1) is therefore the first pass itself;
    * an undecided point with a strong dependency on a C point becomes F; then,
      while points are undecided: every undecided point whose measure exceeds
      the measures of all its undecided strong neighbours (S_i and S^T_i) is C
      (the independent set), and the F marking repeats.  (Measures are
      distinct with probability one; a round that selects nothing takes the
      undecided point of largest (measure, -i) -- a guard hypre does not need.)"""
    if n == 0 or part is None or np.all(np.asarray(part) == np.asarray(part)[0]):
        return np.asarray(cf).copy()  # one partition: no boundary points
    rows, cols = _pattern(S, n)
    lam = np.bincount(cols, minlength=n).astype(np.float64)
    part = np.zeros(n, dtype=np.int64) if part is None else np.asarray(part, dtype=np.int64)
    starts = np.flatnonzero(np.r_[True, part[1:] != part[:-1]])
    ends = np.r_[starts[1:], n]
    rnd = np.empty(n, dtype=np.float64)
    for a, b in zip(starts.tolist(), ends.tolist()):
        rnd[a:b] = hypre_rand(2747 + int(part[a]), b - a)
    measure = lam + rnd
    boundary = np.zeros(n, dtype=bool)
    boundary[rows[part[rows] != part[cols]]] = True
    state = np.where(boundary, U, np.asarray(cf)).astype(np.int64)
    state[(state == U) & (lam == 0)] = F
    Sm = sp.csr_matrix((np.ones(rows.size), (rows, cols)), shape=(n, n))
    sym = (Sm + Sm.T).tocsr()
    sym.sort_indices()
    nonempty = np.diff(sym.indptr) > 0
    starts_nb = sym.indptr[:-1][nonempty]

    def mark_f():
        hasc = (Sm @ (state == C).astype(np.float64)) > 0
        state[(state == U) & hasc] = F

    mark_f()
    while np.any(state == U):
        und = state == U
        m = np.where(und[sym.indices], measure[sym.indices], -1.0)
        nbmax = np.full(n, -1.0)
        if m.size:
            nbmax[nonempty] = np.maximum.reduceat(m, starts_nb)
        sel = und & (measure > nbmax)
        if not sel.any():
            cand = np.flatnonzero(und)
            sel[cand[np.argmax(measure[cand])]] = True
        state[sel] = C
        mark_f()
    return np.where(state == C, C, F).astype(np.int64)


def coarsen(S, n, aggressive, num_paths, part=None):
    """C/F splitting (HMIS = the Ruge-Stueben first pass inside every
    partition, then the PMIS stage, ``pmis_stage``).  part: the level's
    partition, hypre's processes (pls.hypre_ranks) or libpls's automatic
    partitions (levels of >= 2 x 65,536 rows cut into partitions of at least
    that size whose boundaries cut <= 2 % of the strong connections,
    pls.hypre_coarsen_*, so the first pass runs on host threads; the result
    is then BoomerAMG's HMIS with that many processes) -- None: one process."""
    cf = pmis_stage(S, n, rs_partitioned(S, n, part), part)
    if aggressive:
        S2, cpts = second_strength(S, cf, num_paths)
        p2 = None if part is None else part[cpts]
        cf2 = pmis_stage(S2, len(cpts), rs_partitioned(S2, len(cpts), p2), p2)
        cf = np.full(n, F, dtype=np.int64)
        cf[cpts[cf2 == C]] = C
    return cf


def _csr_from_rows(rows, ncols):
    rp, ci, v = [0], [], []
    for row in rows:
        for j in sorted(row):
            if row[j] != 0.0:
                ci.append(j)
                v.append(row[j])
        rp.append(len(ci))
    return sp.csr_matrix((np.asarray(v, dtype=np.float64), np.asarray(ci, dtype=np.int64),
                          np.asarray(rp, dtype=np.int64)), shape=(len(rows), ncols))


def multipass_interp(A, S, cf):
    A, rp, ci, v = _rows(A)
    n = A.shape[0]
    cidx = np.cumsum(cf == C) - 1
    npass = np.where(cf == C, 0, -1)
    order = []
    p = 1
    while True:
        new = [i for i in range(n) if npass[i] < 0 and any(0 <= npass[k] < p for k in S[i].tolist())]
        if not new:
            break
        for i in new:
            npass[i] = p
        order.append(new)
        p += 1
    rows = [dict() for _ in range(n)]
    for i in np.flatnonzero(cf == C).tolist():
        rows[i][int(cidx[i])] = 1.0
    for p, pts in enumerate(order, start=1):
        for i in pts:
            Q = [k for k in S[i].tolist() if 0 <= npass[k] < p]
            qs = set(Q)
            d = 0.0
            neg_all = pos_all = neg_q = pos_q = 0.0
            aik = {}
            for j, a in zip(ci[rp[i]:rp[i + 1]].tolist(), v[rp[i]:rp[i + 1]].tolist()):
                if j == i:
                    d = a
                    continue
                neg_all += min(a, 0.0)
                pos_all += max(a, 0.0)
                if j in qs:
                    aik[j] = a
            for k in Q:
                a = aik.get(k, 0.0)
                neg_q += min(a, 0.0)
                pos_q += max(a, 0.0)
            alpha = beta = 0.0
            if neg_q == 0.0:
                d += neg_all
            else:
                alpha = neg_all / neg_q
            if pos_q == 0.0:
                d += pos_all
            else:
                beta = pos_all / pos_q
            row = {}
            for k in Q:
                a = aik.get(k, 0.0)
                if a == 0.0:
                    continue
                w = -(alpha if a < 0.0 else beta) * a / d
                for j, pv in rows[k].items():
                    row[j] = row.get(j, 0.0) + w * pv
            rows[i] = row
    return _csr_from_rows(rows, int((cf == C).sum()))


def ext_i_interp(A, S, cf):
    A, rp, ci, v = _rows(A)
    n = A.shape[0]
    cidx = np.cumsum(cf == C) - 1
    diag = np.zeros(n)
    for i in range(n):
        for j, a in zip(ci[rp[i]:rp[i + 1]].tolist(), v[rp[i]:rp[i + 1]].tolist()):
            if j == i:
                diag[i] = a
    rows = []
    for i in range(n):
        if cf[i] == C:
            rows.append({int(cidx[i]): 1.0})
            continue
        Si = S[i].tolist()
        sset = set(Si)
        chat = set(j for j in Si if cf[j] == C)
        for k in Si:
            if cf[k] == F:
                chat.update(l for l in S[k].tolist() if cf[l] == C)
        w = {}
        dt = 0.0
        for j, a in zip(ci[rp[i]:rp[i + 1]].tolist(), v[rp[i]:rp[i + 1]].tolist()):
            if j == i:
                dt += a
            elif j in chat:
                w[j] = w.get(j, 0.0) + a
            elif j in sset:
                continue
            else:
                dt += a
        arow = dict(zip(ci[rp[i]:rp[i + 1]].tolist(), v[rp[i]:rp[i + 1]].tolist()))
        for k in Si:
            if cf[k] != F:
                continue
            a_ik = arow[k]
            dk = diag[k]
            kc, kv = ci[rp[k]:rp[k + 1]].tolist(), v[rp[k]:rp[k + 1]].tolist()
            D = 0.0
            for l, a in zip(kc, kv):
                if (l in chat or l == i) and a * dk < 0.0:
                    D += a
            if D == 0.0:
                dt += a_ik
                continue
            distribute = a_ik / D  # hypre's ext+i: distribute = a_ik / sum, then distribute * a_kl
            for l, a in zip(kc, kv):
                if a * dk >= 0.0:
                    continue
                if l in chat:
                    w[l] = w.get(l, 0.0) + distribute * a
                elif l == i:
                    dt += distribute * a
        rows.append({int(cidx[j]): -wv / dt for j, wv in w.items()} if dt != 0.0 else {})
    return _csr_from_rows(rows, int((cf == C).sum()))


def truncate(P, pmax):
    if pmax <= 0:
        return P
    P = P.tocsr()
    P.sort_indices()
    rows = []
    for i in range(P.shape[0]):
        cols = P.indices[P.indptr[i]:P.indptr[i + 1]].tolist()
        vals = P.data[P.indptr[i]:P.indptr[i + 1]].tolist()
        if len(cols) <= pmax:
            rows.append(dict(zip(cols, vals)))
            continue
        keep = sorted(range(len(cols)), key=lambda t: (-abs(vals[t]), cols[t]))[:pmax]
        keep.sort()
        tot = 0.0
        for x in vals:
            tot += x
        kept = 0.0
        for t in keep:
            kept += vals[t]
        s = tot / kept if kept != 0.0 else 1.0
        rows.append({cols[t]: vals[t] * s for t in keep})
    return _csr_from_rows(rows, P.shape[1])


def chunk_ids(n, K):
    """Chunk of every row: hypre's OpenMP partition of n rows over K threads
    (par_relax.c relax type 6: size = n / K, the first n % K chunks one row
    longer; K_l = min(K, n) so no chunk is empty)."""
    K = max(1, min(int(K), n))
    q, r = divmod(n, K)
    lens = np.full(K, q, dtype=np.int64)
    lens[:r] += 1
    return np.repeat(np.arange(K, dtype=np.int64), lens)


def rank_sizes(spec, n):
    """Level-0 rank sizes of ``pls.hypre_ranks`` ("G": PETSc's split of n rows over
    G ranks, or "n0,n1,..."): BoomerAMG as it runs under mpirun -np G -- the
    HMIS first pass inside every rank, then the PMIS stage over the ranks'
    boundary points (``pmis_stage``), a coarse level's rank
    owns the C points of its rows, and each rank's rows are cut into its
    threads' chunks (pls.hypre_relax_chunks / G threads per rank).  None: one rank."""
    if spec is None or str(spec) == "":
        return None
    spec = str(spec)
    if "," not in spec:
        G = int(spec)
        if G <= 1:
            return None
        return [n // G + (1 if q < n % G else 0) for q in range(G)]
    sizes = [int(v) for v in spec.split(",")]
    if sum(sizes) != n:
        raise ValueError("pls.hypre_ranks: the rank sizes do not add up to the block's rows")
    return sizes


def level_chunks(n, K, min_rows):
    """Chunks of a level of n rows: K, fewer when a chunk would hold fewer than
    min_rows rows (0: no floor)."""
    if min_rows > 0:
        K = min(K, max(1, n // min_rows))
    return max(1, min(K, n))


def hybrid_sgs_literal(A, b, u, K, points=None):
    """hypre's relax type 6 with K threads, row by row (pure-Python loops: small
    KAT cases only).  points: boolean mask of the rows this pass relaxes (the
    C / F set), None = every row."""
    A = A.tocsr()
    n = A.shape[0]
    cid = chunk_ids(n, K)
    u = np.array(u, dtype=np.float64)
    tmp = u.copy()
    rp, ci, v = A.indptr, A.indices, A.data
    starts = np.flatnonzero(np.r_[True, cid[1:] != cid[:-1]]) if n else []
    for ns in list(starts):
        ne = ns
        while ne < n and cid[ne] == cid[ns]:
            ne += 1
        for rng in (range(ns, ne), range(ne - 1, ns - 1, -1)):
            for i in rng:
                if points is not None and not points[i]:
                    continue
                d, res = 0.0, b[i]
                for k in range(rp[i], rp[i + 1]):
                    j = ci[k]
                    if j == i:
                        d = v[k]
                    else:
                        res -= v[k] * (u[j] if ns <= j < ne else tmp[j])
                if d != 0.0:
                    u[i] = res / d
    return u


def _sgs_factors(A, cid, idx):
    """(D + L, D + U, strict U) of the chunk-block-diagonal part of A restricted to idx."""
    Asub = A if idx is None else A[idx][:, idx]
    c = cid if idx is None else cid[idx]
    Asub = Asub.tocoo()
    keep = c[Asub.row] == c[Asub.col]
    Abd = sp.csr_matrix((Asub.data[keep], (Asub.row[keep], Asub.col[keep])), shape=Asub.shape)
    Abd.sort_indices()
    return sp.tril(Abd).tocsr(), sp.triu(Abd).tocsr(), sp.triu(Abd, k=1).tocsr()


class PCBoomerAMG:
    type = "hypre"

    def __init__(self, A, db=None, prefix=""):
        db = db or {}
        g = lambda k, d, t=str: opt(db, prefix, "pc_hypre_boomeramg_" + k, d, t)  # noqa: E731
        self.theta = g("strong_threshold", 0.25, float)
        self.mu = g("max_row_sum", 0.9, float)
        self.pmax = g("P_max", 0, int)
        self.agg_nl = g("agg_nl", 0, int)
        self.npaths = g("agg_num_paths", 1, int)
        self.K = g("grid_sweeps_all", 1, int)
        self.max_levels = g("max_levels", 25, int)
        self.no_cf = g("no_CF", False, bool)
        coarsen_t = g("coarsen_type", "HMIS")
        interp_t = g("interp_type", "ext+i")
        if coarsen_t not in _SUPPORTED_COARSEN or interp_t not in _SUPPORTED_INTERP:
            raise NotImplementedError(f"boomeramg coarsen_type {coarsen_t} / interp_type {interp_t}")
        if self.K < 1:
            raise ValueError("grid_sweeps_all must be >= 1")
        self.chunks = int(db.get("pls.hypre_relax_chunks", 256))
        self.chunk_rows = int(db.get("pls.hypre_relax_min_rows", 1024))
        # coarsening partition: 1 = none (default: BoomerAMG on one process, np = 1),
        # K > 1 = K equal partitions, 0 = up to pls.hypre_relax_chunks partitions of at
        # least pls.hypre_coarsen_min_rows (65536) rows (an opt-in speed-up of the setup)
        self.coarsen_chunks = int(db.get("pls.hypre_coarsen_chunks", 1))
        self.coarsen_rows = int(db.get("pls.hypre_coarsen_min_rows", 65536))
        if self.chunks < 1 or self.chunk_rows < 0:
            raise ValueError("pls.hypre_relax_chunks must be >= 1, pls.hypre_relax_min_rows >= 0")
        A = A.tocsr()
        A.sort_indices()
        self.levels = []
        parts = rank_sizes(db.get("pls.hypre_ranks"), A.shape[0])
        while A.shape[0] > 9 and len(self.levels) < self.max_levels - 1:
            n = A.shape[0]
            S = strength(A, self.theta, self.mu)
            aggressive = len(self.levels) < self.agg_nl
            part = None
            if parts is not None:
                part = np.repeat(np.arange(len(parts)), parts)
            elif self.coarsen_chunks > 1:
                part = chunk_ids(n, self.coarsen_chunks)
            elif self.coarsen_chunks == 0:
                part = coarsen_partition(S, n, level_chunks(n, self.chunks, self.coarsen_rows))
            cf = coarsen(S, n, aggressive, self.npaths, part)
            nc = int((cf == C).sum())
            if nc == 0 or nc == n:
                break
            P = multipass_interp(A, S, cf) if aggressive else truncate(ext_i_interp(A, S, cf), self.pmax)
            P.sort_indices()
            R = P.T.tocsr()
            R.sort_indices()
            Ac = (R @ (A @ P)).tocsr()
            Ac.sort_indices()
            self.levels.append({"A": A, "P": P, "R": R, "cf": cf, "parts": parts})
            if parts is not None:  # the coarse level's ranks: their C points
                parts = [int(np.count_nonzero(cf[part == q] == C)) for q in range(len(parts))]
            A = Ac
        self.coarse = A
        self.coarse_lu = spla.splu(sp.csc_matrix(A)) if A.shape[0] else None

    def _smoother(self, L):
        """Per relaxation set ("all", or "C" / "F"): its rows and the hybrid SGS factors."""
        if "sgs" not in L:
            A = L["A"]
            if L.get("parts") is None:
                cid = chunk_ids(A.shape[0], level_chunks(A.shape[0], self.chunks, self.chunk_rows))
            else:  # ranks: each rank's rows in its threads' chunks
                T = max(1, self.chunks // len(L["parts"]))
                cid, base = [], 0
                for sz in L["parts"]:
                    if sz:
                        cid.append(base + chunk_ids(sz, level_chunks(sz, T, self.chunk_rows)))
                        base = int(cid[-1][-1]) + 1
                cid = np.concatenate(cid)
            sets = {"all": None} if self.no_cf else {o: np.flatnonzero(L["cf"] == (C if o == "C" else F)) for o in "CF"}
            L["sgs"] = {k: (idx,) + _sgs_factors(A, cid, idx) for k, idx in sets.items()}
        return L["sgs"]

    def _relax(self, L, b, x, order):
        A = L["A"]
        sm = self._smoother(L)
        sets = [sm["all"]] if self.no_cf else [sm[o] for o in order]
        for _ in range(self.K):
            for idx, lo, up, us in sets:
                if idx is not None and not len(idx):
                    continue
                r = b - A @ x
                if idx is not None:
                    r = r[idx]
                d1 = spla.spsolve_triangular(lo, r, lower=True)
                d2 = spla.spsolve_triangular(up, -(us @ d1), lower=False)
                x = x.copy()
                if idx is None:
                    x += d1 + d2
                else:
                    x[idx] += d1 + d2
        return x

    def _vcycle(self, l, b):
        if l == len(self.levels):
            return self.coarse_lu.solve(b) if self.coarse_lu is not None else b.copy()
        L = self.levels[l]
        x = self._relax(L, b, np.zeros_like(b), "CF")
        r = b - L["A"] @ x
        e = self._vcycle(l + 1, L["R"] @ r)
        x = x + L["P"] @ e
        return self._relax(L, b, x, "FC")

    def apply(self, b):
        b = np.asarray(b, dtype=np.float64)
        if b.size == 0:
            return b.copy()
        return self._vcycle(0, b)
