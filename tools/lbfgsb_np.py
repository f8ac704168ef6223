"""(Development tool: tools/nnls_diag.py compares csrc/nnls.hip against it phase by phase;
it reproduces scipy.optimize.fmin_l_bfgs_b to 1e-16 on the NNLS problems, checked there.)
numpy restatement of L-BFGS-B 3.0 (scipy fmin_l_bfgs_b) for min 0.5||A X - B||^2, X >= 0,
variables the flattened (nb, ncols) block.  Lower bound 0 only (nbd = 1)."""
import numpy as np

EPS = np.finfo(float).eps


def fg(A, B, x, shape):
    X = x.reshape(shape)
    diff = A @ X - B
    return 0.5 * np.sum(diff ** 2), (A.T @ diff).ravel()


def projgr(x, g):
    gi = np.where(g < 0, g, np.minimum(x, g))
    return np.max(np.abs(gi)) if gi.size else 0.0


def bmv(col, sy, wt, v):
    # M v with M the 2col x 2col middle matrix; wt = upper Cholesky factor J' of T
    if col == 0:
        return np.zeros(0)
    p = np.zeros(2 * col)
    D = np.diag(sy)[:col]
    p[col] = v[col]
    for i in range(1, col):
        s = 0.0
        for k in range(i):
            s += sy[i, k] * v[k] / sy[k, k]
        p[col + i] = v[col + i] + s
    # solve J p2 = ... : dtrsl(wt, job 11) solves trans(wt) x = b (wt upper) -> lower solve
    p[col:] = _solve_upper_T(wt[:col, :col], p[col:])
    p[:col] = v[:col] / np.sqrt(D)
    p[col:] = _solve_upper(wt[:col, :col], p[col:])
    p[:col] = -p[:col] / np.sqrt(D)
    for i in range(col):
        s = 0.0
        for k in range(i + 1, col):
            s += sy[k, i] * p[col + k] / sy[i, i]
        p[i] += s
    return p


def _solve_upper_T(U, b):
    # U^T x = b, U upper (forward substitution)
    n = len(b)
    x = b.copy()
    for i in range(n):
        s = x[i]
        for k in range(i):
            s -= U[k, i] * x[k]
        x[i] = s / U[i, i]
    return x


def _solve_upper(U, b):
    n = len(b)
    x = b.copy()
    for i in range(n - 1, -1, -1):
        s = x[i]
        for k in range(i + 1, n):
            s -= U[i, k] * x[k]
        x[i] = s / U[i, i]
    return x


def chol_upper(T):
    # T = U^T U, U upper (dpofa)
    n = T.shape[0]
    U = np.zeros_like(T)
    for j in range(n):
        s = 0.0
        for k in range(j):
            t = T[k, j] - sum(U[i, k] * U[i, j] for i in range(k))
            t = t / U[k, k]
            U[k, j] = t
            s += t * t
        s = T[j, j] - s
        if s <= 0:
            return None
        U[j, j] = np.sqrt(s)
    return U


def dcstep(stx, fx, dx, sty, fy, dy, stp, fp, dp, brackt, stpmin, stpmax):
    sgnd = dp * (dx / abs(dx))
    if fp > fx:
        theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp
        s = max(abs(theta), abs(dx), abs(dp))
        gamma = s * np.sqrt((theta / s) ** 2 - (dx / s) * (dp / s))
        if stp < stx:
            gamma = -gamma
        p = (gamma - dx) + theta
        q = ((gamma - dx) + gamma) + dp
        r = p / q
        stpc = stx + r * (stp - stx)
        stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx)
        stpf = stpc if abs(stpc - stx) < abs(stpq - stx) else stpc + (stpq - stpc) / 2.0
        brackt = True
    elif sgnd < 0:
        theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp
        s = max(abs(theta), abs(dx), abs(dp))
        gamma = s * np.sqrt((theta / s) ** 2 - (dx / s) * (dp / s))
        if stp > stx:
            gamma = -gamma
        p = (gamma - dp) + theta
        q = ((gamma - dp) + gamma) + dx
        r = p / q
        stpc = stp + r * (stx - stp)
        stpq = stp + (dp / (dp - dx)) * (stx - stp)
        stpf = stpc if abs(stpc - stp) > abs(stpq - stp) else stpq
        brackt = True
    elif abs(dp) < abs(dx):
        theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp
        s = max(abs(theta), abs(dx), abs(dp))
        gamma = s * np.sqrt(max(0.0, (theta / s) ** 2 - (dx / s) * (dp / s)))
        if stp > stx:
            gamma = -gamma
        p = (gamma - dp) + theta
        q = (gamma + (dx - dp)) + gamma
        r = p / q
        if r < 0 and gamma != 0:
            stpc = stp + r * (stx - stp)
        elif stp > stx:
            stpc = stpmax
        else:
            stpc = stpmin
        stpq = stp + (dp / (dp - dx)) * (stx - stp)
        if brackt:
            stpf = stpc if abs(stpc - stp) < abs(stpq - stp) else stpq
            if stp > stx:
                stpf = min(stp + 0.66 * (sty - stp), stpf)
            else:
                stpf = max(stp + 0.66 * (sty - stp), stpf)
        else:
            stpf = stpc if abs(stpc - stp) > abs(stpq - stp) else stpq
            stpf = min(stpmax, stpf)
            stpf = max(stpmin, stpf)
    else:
        if brackt:
            theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp
            s = max(abs(theta), abs(dy), abs(dp))
            gamma = s * np.sqrt((theta / s) ** 2 - (dy / s) * (dp / s))
            if stp > sty:
                gamma = -gamma
            p = (gamma - dp) + theta
            q = ((gamma - dp) + gamma) + dy
            r = p / q
            stpc = stp + r * (sty - stp)
            stpf = stpc
        elif stp > stx:
            stpf = stpmax
        else:
            stpf = stpmin
    if fp > fx:
        sty, fy, dy = stp, fp, dp
    else:
        if sgnd < 0:
            sty, fy, dy = stx, fx, dx
        stx, fx, dx = stp, fp, dp
    return stx, fx, dx, sty, fy, dy, stpf, brackt


class Dcsrch:
    def __init__(self, f, g, stp, ftol, gtol, xtol, stpmin, stpmax):
        self.ftol, self.gtol, self.xtol, self.stpmin, self.stpmax = ftol, gtol, xtol, stpmin, stpmax
        self.brackt = False
        self.stage = 1
        self.finit, self.ginit = f, g
        self.gtest = ftol * g
        self.width = stpmax - stpmin
        self.width1 = self.width / 0.5
        self.stx, self.fx, self.gx = 0.0, f, g
        self.sty, self.fy, self.gy = 0.0, f, g
        self.stmin = 0.0
        self.stmax = stp + 4.0 * stp

    def step(self, f, g, stp):
        """returns (task, stp): task in 'FG', 'CONV', 'WARN'"""
        ftest = self.finit + stp * self.gtest
        if self.stage == 1 and f <= ftest and g >= 0:
            self.stage = 2
        task = 'FG'
        if self.brackt and (stp <= self.stmin or stp >= self.stmax):
            task = 'WARN'
        if self.brackt and self.stmax - self.stmin <= self.xtol * self.stmax:
            task = 'WARN'
        if stp == self.stpmax and f <= ftest and g <= self.gtest:
            task = 'WARN'
        if stp == self.stpmin and (f > ftest or g >= self.gtest):
            task = 'WARN'
        if f <= ftest and abs(g) <= self.gtol * (-self.ginit):
            task = 'CONV'
        if task != 'FG':
            return task, stp
        gt = self.gtest
        if self.stage == 1 and f <= self.fx and f > ftest:
            fm = f - stp * gt
            fxm = self.fx - self.stx * gt
            fym = self.fy - self.sty * gt
            gm = g - gt
            gxm = self.gx - gt
            gym = self.gy - gt
            (self.stx, fxm, gxm, self.sty, fym, gym, stp, self.brackt) = dcstep(
                self.stx, fxm, gxm, self.sty, fym, gym, stp, fm, gm, self.brackt, self.stmin, self.stmax)
            self.fx = fxm + self.stx * gt
            self.fy = fym + self.sty * gt
            self.gx = gxm + gt
            self.gy = gym + gt
        else:
            (self.stx, self.fx, self.gx, self.sty, self.fy, self.gy, stp, self.brackt) = dcstep(
                self.stx, self.fx, self.gx, self.sty, self.fy, self.gy, stp, f, g, self.brackt,
                self.stmin, self.stmax)
        if self.brackt:
            if abs(self.sty - self.stx) >= 0.66 * self.width1:
                stp = self.stx + 0.5 * (self.sty - self.stx)
            self.width1 = self.width
            self.width = abs(self.sty - self.stx)
        if self.brackt:
            self.stmin = min(self.stx, self.sty)
            self.stmax = max(self.stx, self.sty)
        else:
            self.stmin = stp + 1.1 * (stp - self.stx)
            self.stmax = stp + 4.0 * (stp - self.stx)
        stp = max(stp, self.stpmin)
        stp = min(stp, self.stpmax)
        if (self.brackt and (stp <= self.stmin or stp >= self.stmax)) or (
                self.brackt and self.stmax - self.stmin <= self.xtol * self.stmax):
            stp = self.stx
        return 'FG', stp


def lbfgsb(A, B, x0, m=None, factr=1e7, pgtol=1e-5, maxiter=15000, maxls=20, trace=None, snap=None):
    shape = x0.shape
    x = np.array(x0, dtype=np.float64).ravel()
    n = x.size
    A = np.asarray(A)
    m = A.shape[1] if m is None else m
    tol = factr * EPS
    WS = np.zeros((0, n))
    WY = np.zeros((0, n))
    sy = np.zeros((0, 0))
    ss = np.zeros((0, 0))
    wt = None
    theta = 1.0
    col = 0
    updatd = False
    iwhere = np.zeros(n, np.int32)  # active(): x0 >= 0, nbd = 1 -> 0
    x = np.maximum(x, 0.0)
    f, g = fg(A, B, x, shape)
    nfev = 1
    sbgnrm = projgr(x, g)
    it = 0
    if sbgnrm <= pgtol:
        return x.reshape(shape), dict(nit=0, task='CONV_PGTOL')
    while True:
        # ---------------- cauchy ----------------
        neggi = -g
        xlower = x <= 0.0
        iwhere = np.zeros(n, np.int32)
        iwhere[xlower & (neggi <= 0)] = 1
        iwhere[(~xlower) & (np.abs(neggi) <= 0)] = -3
        moving = (iwhere == 0)
        d = np.where(moving, neggi, 0.0)
        f1 = -np.sum(d * d)  # order differs
        p = np.concatenate([WY @ d, WS @ d]) if col else np.zeros(0)
        bkpt = moving & (neggi < 0)
        tb = np.where(bkpt, x / np.where(bkpt, -neggi, 1.0), np.inf)
        nbreak = int(bkpt.sum())
        nfree_cnt = int((moving & ~bkpt).sum())
        bnded = not np.any(moving & ~bkpt & (np.abs(neggi) > 0))
        if col:
            p[col:] *= theta
        xcp = x.copy()
        c = np.zeros(2 * col)
        nseg = 0
        if nbreak == 0 and nfree_cnt == 0:
            pass  # d = 0
        else:
            f2 = -theta * f1
            f2_org = f2
            if col:
                v = bmv(col, sy, wt, p)
                f2 = f2 - v @ p
            dtm = -f1 / f2
            tsum = 0.0
            nseg = 1
            order = np.argsort(tb[bkpt], kind='stable')
            idx = np.nonzero(bkpt)[0][order]
            tj = 0.0
            done999 = False
            k = 0
            while k < nbreak:
                tj0 = tj
                ibp = idx[k]
                tj = tb[ibp]
                dt = tj - tj0
                if dtm < dt:
                    break
                tsum += dt
                k += 1
                dibp = d[ibp]
                d[ibp] = 0.0
                zibp = 0.0 - x[ibp]
                xcp[ibp] = 0.0
                iwhere[ibp] = 1
                if k == nbreak and nbreak == n:
                    dtm = dt
                    done999 = True
                    break
                nseg += 1
                dibp2 = dibp * dibp
                f1 = f1 + dt * f2 + dibp2 - theta * dibp * zibp
                f2 = f2 - theta * dibp2
                if col:
                    c = c + dt * p
                    wbp = np.concatenate([WY[:, ibp], theta * WS[:, ibp]])
                    v = bmv(col, sy, wt, wbp)
                    wmc = c @ v
                    wmp = p @ v
                    wmw = wbp @ v
                    p = p - dibp * wbp
                    f1 = f1 + dibp * wmc
                    f2 = f2 + 2.0 * dibp * wmp - dibp2 * wmw
                f2 = max(EPS * f2_org, f2)
                if k < nbreak:
                    dtm = -f1 / f2
                elif bnded:
                    f1 = f2 = dtm = 0.0
                else:
                    dtm = -f1 / f2
            if not done999:
                if dtm <= 0:
                    dtm = 0.0
                tsum += dtm
                xcp = xcp + tsum * d  # d is zero at fixed breakpoints; xcp there is 0
                # careful: daxpy adds tsum*d to every entry incl. the passed ones (d=0 there)
            if col:
                c = c + dtm * p
        if snap is not None and it in snap:
            snap[it].update(xcp=xcp.copy(), c=c.copy(), p=p.copy(), iwhere=iwhere.copy(), theta=theta,
                            col=col, tsum=locals().get('tsum', 0.0), nbreak=nbreak)
        # ---------------- freev ----------------
        free = iwhere <= 0
        nfree = int(free.sum())
        # ---------------- formk / cmprlb / subsm ----------------
        z = xcp
        if nfree > 0 and col > 0:
            fi = np.nonzero(free)[0]
            ai = np.nonzero(~free)[0]
            WYf, WSf = WY[:, fi], WS[:, fi]
            WYa, WSa = WY[:, ai], WS[:, ai]
            YY = WYf @ WYf.T
            SSa = WSa @ WSa.T
            SYa = WSa @ WYa.T
            SYf = WSf @ WYf.T
            wn1_21 = np.where(np.arange(col)[:, None] > np.arange(col)[None, :], SYa, SYf)
            wn = np.zeros((2 * col, 2 * col))
            wn[:col, :col] = YY / theta + np.diag(np.diag(sy)[:col])
            wn[col:, col:] = SSa * theta
            # wn(jy, is) upper (1,2) block: for jy < iy: -wn1(is1, jy); jy >= iy: wn1(is1, jy)
            for iy in range(col):
                for jy in range(col):
                    wn[jy, col + iy] = -wn1_21[iy, jy] if jy < iy else wn1_21[iy, jy]
            U11 = chol_upper(wn[:col, :col])
            if U11 is None:
                raise RuntimeError('formk info -1')
            wn_f = np.zeros_like(wn)
            wn_f[:col, :col] = U11
            for js in range(col, 2 * col):
                wn_f[:col, js] = _solve_upper_T(U11, wn[:col, js])
            W22 = wn[col:, col:].copy()
            for i in range(col):
                for j in range(i, col):
                    W22[i, j] += wn_f[:col, col + i] @ wn_f[:col, col + j]
            W22 = np.triu(W22) + np.triu(W22, 1).T
            U22 = chol_upper(W22)
            if U22 is None:
                raise RuntimeError('formk info -2')
            wn_f[col:, col:] = U22
            # cmprlb
            wa = bmv(col, sy, wt, c)
            r = -theta * (z[fi] - x[fi]) - g[fi]
            r = r + WYf.T @ wa[:col] + WSf.T @ (theta * wa[col:])
            # subsm
            wv = np.concatenate([WYf @ r, theta * (WSf @ r)])
            if snap is not None and it in snap:
                rr_full = np.zeros(n)
                rr_full[fi] = r
                snap[it].update(r=rr_full, wv_raw=wv.copy(), wa=wa.copy(), wn=wn.copy(), wn_f=wn_f.copy())
            wv = _solve_upper_T(wn_f, wv)
            wv[:col] = -wv[:col]
            wv = _solve_upper(wn_f, wv)
            dd = r + WYf.T @ (wv[:col] / theta) + WSf.T @ wv[col:]
            dd = dd / theta
            xp = z.copy()
            zk = z[fi] + dd
            znew = np.maximum(0.0, zk)
            iword = bool(np.any(znew == 0.0))
            z = z.copy()
            z[fi] = znew
            if iword:
                dd_p = np.sum((z - x) * g)
                if dd_p > 0:
                    z = xp.copy()
                    alpha = 1.0
                    temp1 = alpha
                    ibd = -1
                    for ii, k in enumerate(fi):
                        dk = dd[ii]
                        if dk < 0:
                            temp2 = 0.0 - z[k]
                            if temp2 >= 0:
                                temp1 = 0.0
                            elif dk * alpha < temp2:
                                temp1 = temp2 / dk
                        if temp1 < alpha:
                            alpha = temp1
                            ibd = ii
                    if alpha < 1.0:
                        dk = dd[ibd]
                        k = fi[ibd]
                        if dk < 0:
                            z[k] = 0.0
                            dd[ibd] = 0.0
                    z[fi] = z[fi] + alpha * dd
                    if trace is not None:
                        trace.append(('backtrack', it, alpha))
        if snap is not None and it in snap:
            snap[it].update(z=z.copy())
        # ---------------- line search ----------------
        d = z - x
        dtd = d @ d
        dnorm = np.sqrt(dtd)
        if it == 0:
            stpmx = 1.0
        else:
            stpmx = 1e10
            neg = d < 0
            if np.any(neg):
                a2 = 0.0 - x[neg]
                a1 = d[neg]
                if np.any(a2 >= 0):
                    stpmx = 0.0
                else:
                    # sequential: if a1*stpmx < a2: stpmx = a2/a1
                    for aa1, aa2 in zip(a1, a2):
                        if aa1 * stpmx < aa2:
                            stpmx = aa2 / aa1
        stp = min(1.0 / dnorm, stpmx) if it == 0 else 1.0
        t = x.copy()
        r_old = g.copy()
        fold = f
        gd = g @ d
        gdold = gd
        if gd >= 0:
            raise RuntimeError('ascent direction')
        ls = Dcsrch(f, gd, stp, 1e-3, 0.9, 0.1, 0.0, stpmx)
        nls = 0
        while True:
            x = z.copy() if stp == 1.0 else stp * d + t
            f, g = fg(A, B, x, shape)
            nfev += 1
            nls += 1
            gd = g @ d
            task, stp_new = ls.step(f, gd, stp)
            if task != 'FG':
                break
            if nls >= maxls:
                raise RuntimeError('line search limit')
            stp = stp_new
        it += 1
        sbgnrm = projgr(x, g)
        if trace is not None:
            trace.append(('iter', it, f, sbgnrm, nseg, nbreak, col, stp, nls, nfree))
        if sbgnrm <= pgtol:
            return x.reshape(shape), dict(nit=it, task='CONV_PGTOL', nfev=nfev)
        if it >= maxiter:
            return x.reshape(shape), dict(nit=it, task='MAXITER', nfev=nfev)
        ddum = max(abs(fold), abs(f), 1.0)
        if (fold - f) <= tol * ddum:
            return x.reshape(shape), dict(nit=it, task='CONV_FACTR', nfev=nfev)
        rvec = g - r_old
        rr = rvec @ rvec
        if stp == 1.0:
            dr = gd - gdold
            ddum = -gdold
        else:
            dr = (gd - gdold) * stp
            d = stp * d
            ddum = -gdold * stp
        if dr <= EPS * ddum:
            updatd = False
            if trace is not None:
                trace.append(('skip', it))
            continue
        updatd = True
        if col == m:
            raise RuntimeError('memory wrap not restated')
        WS = np.vstack([WS, d[None]])
        WY = np.vstack([WY, rvec[None]])
        col += 1
        theta = rr / dr
        sy_n = np.zeros((col, col))
        ss_n = np.zeros((col, col))
        sy_n[:col - 1, :col - 1] = sy
        ss_n[:col - 1, :col - 1] = ss
        for j in range(col - 1):
            sy_n[col - 1, j] = d @ WY[j]
            ss_n[j, col - 1] = WS[j] @ d
        ss_n[col - 1, col - 1] = dtd if stp == 1.0 else stp * stp * dtd
        sy_n[col - 1, col - 1] = dr
        sy, ss = sy_n, ss_n
        # formt
        T = np.zeros((col, col))
        for j in range(col):
            T[0, j] = theta * ss[0, j]
        for i in range(1, col):
            for j in range(i, col):
                k1 = min(i, j)
                ddum2 = 0.0
                for k in range(k1):
                    ddum2 += sy[i, k] * sy[j, k] / sy[k, k]
                T[i, j] = ddum2 + theta * ss[i, j]
        T = np.triu(T) + np.triu(T, 1).T
        wt = chol_upper(T)
        if wt is None:
            raise RuntimeError('formt info')
