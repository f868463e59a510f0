"""Lab: thread-level numpy emulation of svd_tri.h's lower-triangle tridiagonalisation stages
(s3_stage<TR, NT>), to check the tile / grid / reduce bookkeeping for a workgroup size on the host:
the eigenvalues of the tridiagonal it produces against numpy's of G.

    python3 tools/lab/tri_s3_emul.py [NT] [C]
"""
import sys

import numpy as np


def tri_cum(c, nb):
    return c * (nb - c)


def tri_off(r, nb):
    m, e = r >> 1, r & 1
    return 2 * nb * m - m * (m - 1) + e * (nb - m)


def tri_map(t, tr, nt):
    tc, q, nb = 2 * tr, tr * tr, 32 if nt == 256 else 64
    c = 0
    while c < nb // 2 - 1 and tri_cum(c + 1, nb) <= t:
        c += 1
    cb, r = c, 2 * c + 1 + (t - tri_cum(c, nb))
    last = tc * cb + tc - 1
    dr, dc = [-1, -1], [-1, -1]
    prev, ovf = -q, 0
    for b in range(nb // 2):
        a = (tri_cum(b, nb) + q - 1) // q * q
        a = max(a, prev + q)
        slot = 0
        if a + q > nt:
            a = nt - 64 + q * ovf
            ovf += 1
            slot = 1
        else:
            prev = a
        if a <= t < a + q:
            u = t - a
            dr[slot], dc[slot] = 2 * b * tr + u // tr, 2 * b * tr + u % tr
            last = max(last, 2 * b * tr + tr - 1)
    return r, cb, dr, dc, last


class State:
    def __init__(self, C):
        self.C = C
        self.vec = np.zeros((136, 3), complex)  # v, p, z
        self.gk1 = np.zeros(128, complex)
        self.scal = np.zeros(2, complex)
        self.ktp = None
        self.d = np.zeros(128)
        self.e = np.zeros(128)
        self.tau = np.zeros(130, complex)  # tau[k + 1]
        self.scratch = None


def stage(st, G, tr, nt, k0, k1, mode):
    C = st.C
    nb = 32 if nt == 256 else 64
    nw = nt // 64
    tc, S = 2 * tr, nb * tr
    gpr = nt // S
    base = 128 - S
    maps = [tri_map(t, tr, nt) for t in range(nt)]
    wlast = [max(maps[t][4] for t in range(64 * w, 64 * w + 64)) for w in range(nw)]

    def ld(r, c):
        if mode == 2:
            if r >= C or c >= C:
                return 0j
            return G[r, c]
        a, b = r - base, c - base
        return st.scratch[a, b] if r >= c else np.conj(st.scratch[b, a])

    tiles, gds = [], []
    for t in range(nt):
        R, Cb, dr, dc, _ = maps[t]
        rl0, cl0 = base + tr * R, base + tc * Cb
        tiles.append(np.array([[ld(rl0 + i, cl0 + jj) for jj in range(tc)] for i in range(tr)], complex))
        gds.append([ld(base + dr[s], base + dc[s]) if dr[s] >= 0 else 0j for s in range(2)])
    if mode == 2:
        st.vec[:] = 0
        st.ktp = np.zeros(nw, complex)
        st.tau[0] = 0
        for t in range(nt):
            R, Cb, dr, dc, _ = maps[t]
            rl0, cl0 = base + tr * R, base + tc * Cb
            if cl0 == 0:
                for i in range(tr):
                    if rl0 + i > 0:
                        st.vec[rl0 + i, 2] = tiles[t][i, 0]
            for s in range(2):
                a, b = base + dr[s], base + dc[s]
                if dr[s] >= 0 and b == 0 and a > 0:
                    st.vec[a, 2] = gds[t][s]
    grid_n = tr * tri_off(nb, nb)
    grid = np.full(grid_n, np.nan + 0j)  # (LDS: entries of retired waves keep their last value)
    for k in range(k0, k1):
        kl = k - base
        kt = st.ktp.sum()
        a2 = -0.5 * st.tau[k] * kt  # tau[k - 1]
        pk = st.vec[k, 1]
        s = complex(pk.real + 2 * a2.real, -pk.imag)
        a2r2 = 2 * a2.real
        V = st.vec.copy()
        diag_pr = {}
        for t in range(nt):
            if kl > wlast[t // 64] + 1:
                continue
            R, Cb, dr, dc, _ = maps[t]
            half = R == 2 * Cb + 1
            rl0, cl0 = base + tr * R, base + tc * Cb
            g = tiles[t]
            yr = np.zeros(tr, complex)
            vr = V[rl0:rl0 + tr, 0]
            wr = V[rl0:rl0 + tr, 1] + a2r2 * vr
            for jj in range(tc):
                c = cl0 + jj
                vc, pc, zc = V[c]
                xc = (zc - s * vc) if c > k else 0j
                for i in range(tr):
                    g[i, jj] -= vr[i] * np.conj(pc) + wr[i] * np.conj(vc)
                    yr[i] += g[i, jj] * xc
                if c == k + 1:
                    for i in range(tr):
                        if rl0 + i >= k + 1:
                            st.gk1[rl0 + i] = g[i, jj]
                if jj >= tr and c == k:
                    for i in range(tr):
                        if rl0 + i == k:
                            st.d[k] = g[i, jj].real
            o_row = tr * (tri_off(R, nb) + Cb)
            o_clo = tr * (tri_off(2 * Cb, nb) + R - Cb - 1)
            o_chi = tr * (tri_off(2 * Cb + 1, nb) + R - Cb)
            grid[o_row:o_row + tr] = yr
            xr = np.array([(V[rl0 + i, 2] - s * V[rl0 + i, 0]) if rl0 + i > k else 0j for i in range(tr)])
            for jj in range(tc):
                yc = np.sum(np.conj(g[:, jj]) * xr)
                if jj < tr:
                    grid[o_clo + jj] = yc
                else:
                    grid[o_chi + jj - tr] = 0j if half else yc
            for sl in range(2):
                if sl == 1 and t // 64 != nw - 1:
                    continue
                if dr[sl] < 0:
                    continue
                rd, cd = base + dr[sl], base + dc[sl]
                v, p = V[rd, 0], V[rd, 1]
                w = p + a2r2 * v
                vc, pc, zc = V[cd]
                xc = (zc - s * vc) if cd > k else 0j
                gds[t][sl] -= v * np.conj(pc) + w * np.conj(vc)
                tt = gds[t][sl]
                diag_pr.setdefault((sl, rd), []).append((cd, tt * xc))
                if cd == k + 1 and rd >= k + 1:
                    st.gk1[rd] = tt
                if rd == k and cd == k:
                    st.d[k] = tt.real
                if cd % tr == 0:
                    B = dr[sl] // (2 * tr)
                    od = tr * (tri_off(2 * B, nb) + nb - 1 - B) + (dr[sl] - 2 * B * tr)
                    diag_pr[(sl, rd, 'o')] = od
        for key, val in list(diag_pr.items()):
            if len(key) == 2:
                grid[diag_pr[(key[0], key[1], 'o')]] = sum(x for _, x in val)
        # zlarfg (wave 0)
        xs = np.array([(V[r, 2] - s * V[r, 0]) for r in range(128)])
        xn2 = sum(abs(xs[r]) ** 2 for r in range(128) if r > k + 1)
        alpha = xs[k + 1]
        x2 = abs(alpha) ** 2 + xn2
        nn = np.sqrt(x2)
        triv = xn2 == 0.0 and alpha.imag == 0.0
        beta = alpha.real if triv else (-nn if alpha.real >= 0 else nn)
        tau = 0j if triv else complex((beta - alpha.real) / beta, -alpha.imag / beta)
        scl = 0j if triv else 1.0 / (alpha - beta)
        st.tau[k + 1] = tau
        st.e[k] = beta
        ts = tau * scl
        # reduce
        newv = st.vec.copy()
        kt = np.zeros(nw, complex)
        for rloc in range(S):
            Rr, ir = rloc // tr, rloc % tr
            n = nb - (Rr >> 1)
            offs = [tr * tri_off(Rr, nb) + ir + tr * o for o in range(n)]
            vals = grid[offs]
            assert not np.any(np.isnan(vals.real)), (k, rloc, [o for o, v in zip(offs, vals) if np.isnan(v.real)][:4])
            y = vals.sum()
            r = base + rloc
            g1 = st.gk1[r]
            ssum = y - beta * g1
            rowact, below = k < r < C, k + 1 < r < C
            p = ts * ssum if rowact else 0j
            v = (V[r, 2] - s * V[r, 0]) * scl if below else (1.0 + 0j if r == k + 1 else 0j)
            z = g1 - p if below else 0j
            newv[r] = (v, p, z)
            if rowact:
                st.hh[(k, r)] = v
            wv = (rloc * gpr) // 64
            kt[wv] += np.conj(p) * v
        st.vec = newv
        st.ktp = kt
    if k1 < C - 1:
        nbb, SN = base + S // 2, S // 2
        sc = np.zeros((SN, SN), complex)
        for t in range(nt):
            R, Cb, dr, dc, _ = maps[t]
            rl0, cl0 = base + tr * R, base + tc * Cb
            for i in range(tr):
                for jj in range(tc):
                    r, c = rl0 + i, cl0 + jj
                    if c >= nbb and r >= c:
                        sc[r - nbb, c - nbb] = tiles[t][i, jj]
            for sl in range(2):
                r, c = base + dr[sl], base + dc[sl]
                if dr[sl] >= 0 and c >= nbb and r >= c:
                    sc[r - nbb, c - nbb] = gds[t][sl]
        st.scratch = sc
    else:
        kk = C - 1
        a2 = -0.5 * st.tau[kk] * st.ktp.sum()
        v, p = st.vec[kk, 0], st.vec[kk, 1]
        w = a2 * v + p
        upd = 2.0 * (v.real * w.real + v.imag * w.imag)
        for t in range(nt):
            R, Cb, dr, dc, _ = maps[t]
            rl0, cl0 = base + tr * R, base + tc * Cb
            for i in range(tr):
                for jj in range(tr, tc):
                    if rl0 + i == kk and cl0 + jj == kk:
                        st.d[kk] = tiles[t][i, jj].real - upd
            for sl in range(2):
                r, c = base + dr[sl], base + dc[sl]
                if dr[sl] >= 0 and r == kk and c == kk:
                    st.d[kk] = gds[t][sl].real - upd


def main():
    nt = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    rng = np.random.default_rng(3)
    X = rng.standard_normal((C, C)) + 1j * rng.standard_normal((C, C))
    G = X.conj().T @ X
    st = State(C)
    st.hh = {}
    kend = C - 1
    if nt == 1024:
        stage(st, G, 2, 1024, 0, min(kend, 64), 2)
        if kend > 64:
            stage(st, G, 1, 1024, 64, kend, 1)
    else:
        stage(st, G, 4, 256, 0, min(kend, 64), 2)
        if kend > 64:
            stage(st, G, 2, 256, 64, min(kend, 96), 1)
        if kend > 96:
            stage(st, G, 1, 256, 96, kend, 1)
    T = np.diag(st.d[:C]) + np.diag(st.e[:C - 1], 1) + np.diag(st.e[:C - 1], -1)
    ev = np.sort(np.linalg.eigvalsh(T))
    ref = np.sort(np.linalg.eigvalsh(G))
    print(f"NT={nt} C={C}: max |eig(T) - eig(G)| / ||G|| = {np.max(np.abs(ev - ref)) / ref[-1]:.2e}")


if __name__ == "__main__":
    main()
