"""pyref -- an independent pure-Python restatement of the reference shaders (TEST INFRASTRUCTURE).

Written directly from the GLSL (VDIGenerator.comp, AccumulateVDI.comp, VolumeRaycaster.comp,
AccumulatePlainImage.comp, PlainImageCompositor.comp) and the numerical contract in DESIGN.md,
without sharing code with oracle/insitu_oracle.c.  It is slow (pure Python, binary32 emulated
with correctly rounded double arithmetic) and exists to pin the C oracle on small cases: the
two restatements must agree bit for bit.  It also generates the committed golden fixtures
(tests/golden/make_golden.py).

binary32 emulation: for +,-,*,/ and sqrt, computing in double and rounding once to binary32 is
exact (53 >= 2*24+2, no double-rounding error); fused multiply-add needs the explicit tie
correction in fma32().
"""
from __future__ import annotations

import math
import struct

_pack, _unpack = struct.Struct("<f").pack, struct.Struct("<f").unpack
_packI, _unpackI = struct.Struct("<I").pack, struct.Struct("<I").unpack


def r32(x: float) -> float:
    """round a double to the nearest binary32 (ties to even)"""
    try:
        return _unpack(_pack(x))[0]
    except OverflowError:
        return math.copysign(math.inf, x)


def bits(x: float) -> int:
    return _unpackI(_pack(x))[0]


def from_bits(u: int) -> float:
    return _unpack(_packI(u & 0xFFFFFFFF))[0]


def add(a, b): return r32(a + b)
def sub(a, b): return r32(a - b)
def mul(a, b): return r32(a * b)
def div(a, b):
    if b == 0.0:
        if a == 0.0 or a != a:
            return math.nan
        return math.copysign(math.inf, a) * math.copysign(1.0, b)
    return r32(a / b)
def sqrt32(a): return r32(math.sqrt(a)) if a >= 0 else math.nan


def _next32(x: float, toward: float) -> float:
    u = bits(x)
    if x == 0.0:
        return from_bits(1) if toward > 0 else from_bits(0x80000001)
    up = (toward > x) == (x > 0)
    return from_bits(u + 1 if up else u - 1)


def fma32(a: float, b: float, c: float) -> float:
    """correctly rounded binary32 fma(a,b,c) for binary32 inputs"""
    p = a * b                     # exact in double (24+24 bits)
    s = p + c
    if math.isinf(s) or math.isnan(s):
        return r32(s)
    bb = s - p
    err = (p - (s - bb)) + (c - bb)   # TwoSum: p + c == s + err exactly
    r = r32(s)
    if err != 0.0 and r != s and not math.isinf(r):
        o = _next32(r, s)
        if (r + o) / 2.0 == s:        # s sits exactly on a binary32 tie: err decides
            hi, lo = (r, o) if r > o else (o, r)
            r = hi if err > 0 else lo
    return r


def gmin(x, y): return y if y < x else x
def gmax(x, y): return y if x < y else x
def mix(x, y, a): return fma32(y, a, mul(x, sub(1.0, a)))


def matvec(m, v):
    """GLSL mat4*vec4, m column-major list of 16 binary32"""
    out = []
    for r in range(4):
        t = mul(m[r], v[0])
        t = fma32(m[4 + r], v[1], t)
        t = fma32(m[8 + r], v[2], t)
        out.append(fma32(m[12 + r], v[3], t))
    return out


def matmul(a, b):
    out = [0.0] * 16
    for c in range(4):
        col = matvec(a, b[4 * c:4 * c + 4])
        out[4 * c:4 * c + 4] = col
    return out


def length(v):
    t = mul(v[0], v[0])
    for k in range(1, len(v)):
        t = fma32(v[k], v[k], t)
    return sqrt32(t)


def vsub(a, b): return [sub(x, y) for x, y in zip(a, b)]
def vmix(a, b, t): return [mix(x, y, t) for x, y in zip(a, b)]
def divide_w(v):
    r = div(1.0, v[3])
    return [mul(x, r) for x in v]


# --------------------------------------------------------------- deterministic pow (contract)
def log2_32(x: float) -> float:
    if x != x or x < 0.0:
        return math.nan
    if x == 0.0:
        return -math.inf
    if math.isinf(x):
        return math.inf
    eadj = 0
    if x < 1.17549435e-38:
        x = mul(x, 8388608.0)
        eadj = -23
    u = bits(x)
    e = ((u >> 23) & 0xFF) - 127 + eadj
    m = from_bits((u & 0x007FFFFF) | 0x3F800000)
    if m > r32(1.41421354):
        m = mul(m, 0.5)
        e += 1
    f = sub(m, 1.0)
    s = div(f, add(2.0, f))
    z = mul(s, s)
    p = fma32(z, r32(0.0909090936), r32(0.111111112))
    p = fma32(z, p, r32(0.142857149))
    p = fma32(z, p, r32(0.200000003))
    p = fma32(z, p, r32(0.333333343))
    s2 = add(s, s)
    ln = fma32(mul(s2, z), p, s2)
    return fma32(ln, r32(1.44269502), float(e))


_EXP2_C = [r32(c) for c in (1.52527336e-05, 1.54035297e-04, 1.33335581e-03, 9.61812911e-03, 5.55041087e-02,
                            2.40226507e-01, 6.93147182e-01, 1.0)]


def exp2_32(y: float) -> float:
    if y != y:
        return y
    if y >= 128.0:
        return math.inf
    if y < -150.0:
        return 0.0
    n = float(round(y))      # Python round = ties to even = rintf
    f = sub(y, n)
    p = _EXP2_C[0]
    for c in _EXP2_C[1:]:
        p = fma32(p, f, c)
    ni = int(n)
    if ni > 127:
        return mul(mul(p, from_bits(0x7F000000)), 2.0)
    if ni >= -126:
        return mul(p, from_bits((ni + 127) << 23))
    return mul(mul(p, from_bits((ni + 127 + 64) << 23)), from_bits((127 - 64) << 23))


def pow32(x, y): return exp2_32(mul(y, log2_32(x)))
def adjust_opacity(a, l): return sub(1.0, pow32(sub(1.0, a), l))   # VDIGenerator.comp:80-82


def unorm8(x):
    q = (x if x < 1.0 else 1.0) if x > 0.0 else 0.0
    return int(math.floor(fma32(q, 255.0, 0.5)))


# --------------------------------------------------------------- scenery sampleVolume (contract)
class Volume:
    def __init__(self, data, dims, im, tf, cmap, conv_k, conv_off):
        """data: flat sequence of raw voxel values (x fastest), dims (nx,ny,nz), im column-major;
        tf: list of alpha texels; cmap: list of (r,g,b,a) texels."""
        self.data = [float(v) for v in data]
        self.dims = dims
        self.im = [r32(v) for v in im]
        self.tf = [r32(v) for v in tf]
        self.cmap = [[r32(c) for c in t] for t in cmap]
        self.k = r32(conv_k)
        self.off = r32(conv_off)

    @staticmethod
    def _pair(t, n):
        fl = math.floor(t) if t == t else math.nan
        frac = sub(t, fl) if fl == fl else math.nan
        if not (fl >= -1.0):
            fl = -1.0
        if fl > n:
            fl = float(n)
        i = int(fl)
        return min(max(i, 0), n - 1), min(max(i + 1, 0), n - 1), frac

    def voxel(self, x, y, z):
        nx, ny, _ = self.dims
        return self.data[(z * ny + y) * nx + x]

    def sample(self, wpos):
        p = matvec(self.im, wpos)
        nx, ny, nz = self.dims
        x0, x1, fx = self._pair(p[0], nx)
        y0, y1, fy = self._pair(p[1], ny)
        z0, z1, fz = self._pair(p[2], nz)
        v = self.voxel
        c00 = mix(v(x0, y0, z0), v(x1, y0, z0), fx)
        c10 = mix(v(x0, y1, z0), v(x1, y1, z0), fx)
        c01 = mix(v(x0, y0, z1), v(x1, y0, z1), fx)
        c11 = mix(v(x0, y1, z1), v(x1, y1, z1), fx)
        val = mix(mix(c00, c10, fy), mix(c01, c11, fy), fz)
        s = add(fma32(val, self.k, self.off), r32(0.001))
        i0, i1, fr = self._pair(fma32(s, float(len(self.tf)), -0.5), len(self.tf))
        a = mix(self.tf[i0], self.tf[i1], fr)
        i0, i1, fr = self._pair(fma32(s, float(len(self.cmap)), -0.5), len(self.cmap))
        c0, c1 = self.cmap[i0], self.cmap[i1]
        return [mix(c0[0], c1[0], fr), mix(c0[1], c1[1], fr), mix(c0[2], c1[2], fr), a]

    def intersect(self, wfront, wback):
        """intersectBox(im*wfront, im*wback - im*wfront, 0, dims)  (VDIGenerator.comp:64-78)"""
        mf, mb = matvec(self.im, wfront), matvec(self.im, wback)
        tmin, tmax = [], []
        for k in range(3):
            ro, rd = mf[k], sub(mb[k], mf[k])
            inv = div(1.0, rd)
            tbot = mul(inv, sub(0.0, ro))
            ttop = mul(inv, sub(float(self.dims[k]), ro))
            tmin.append(gmin(ttop, tbot))
            tmax.append(gmax(ttop, tbot))
        return (gmax(gmax(tmin[0], tmin[1]), gmax(tmin[0], tmin[2])),
                gmin(gmin(tmax[0], tmax[1]), gmin(tmax[0], tmax[2])))


def _ray(ipv, gx, gy, W, H):
    uvx = fma32(div(float(gx), float(W)), 2.0, -1.0)
    uvy = fma32(div(float(gy), float(H)), 2.0, -1.0)
    wfront = divide_w(matvec(ipv, [uvx, uvy, -1.0, 1.0]))
    wback = divide_w(matvec(ipv, [uvx, uvy, 1.0, 1.0]))
    return uvx, uvy, wfront, wback


# --------------------------------------------------------------- VDIGenerator + AccumulateVDI
def vdi_pixel(vol: Volume, cam: dict, gx: int, gy: int, W: int, H: int, S: int):
    """Returns (supersegments [(start, end, (r,g,b,a))...] as written, octree cell increments
    [(cx, cy, z)...], passes).  cam: dict of column-major lists view/proj/inv_view/inv_proj + nw, tmax."""
    ipv = matmul(cam["inv_view"], cam["inv_proj"])
    pv = matmul(cam["proj"], cam["view"])
    view = cam["view"]
    nw = r32(cam["nw"])
    ncx, ncy = W // 8, H // 8
    cx = int(math.floor(mul(div(float(gx), float(W)), float(ncx))))
    cy = int(math.floor(mul(div(float(gy), float(H)), float(ncy))))
    interval = div(sub(20.0, r32(0.1)), float(S))
    uvx, uvy, wfront, wback = _ray(ipv, gx, gy, W, H)
    tnear, tfar = 1.0, 0.0
    n, f = vol.intersect(wfront, wback)
    f = gmin(r32(cam["tmax"]), f)
    vis, lnear, lfar = False, 0.0, 0.0
    if n < f:
        lnear, lfar = n, f
        tnear = gmin(tnear, gmax(0.0, n))
        tfar = gmax(tfar, f)
        vis = True
    written, cells = [], []
    passes = 0

    def zcell(z_view):
        q = math.floor(div(abs(sub(z_view, -r32(0.1))), interval))
        return S if not (q < S) else int(q)

    def close(start, end, adj):
        written.append((start, end, tuple(adj)))
        sw = divide_w(matvec(ipv, [uvx, uvy, start, 1.0]))
        ew = divide_w(matvec(ipv, [uvx, uvy, end, 1.0]))
        sc, ec = zcell(matvec(view, sw)[2]), zcell(matvec(view, ew)[2])
        if 0 <= cx < ncx and 0 <= cy < ncy:
            for j in range(sc, min(ec, S - 1) + 1):
                cells.append((cx, cy, j))

    if tnear < tfar:
        num_steps = int(math.trunc(div(sub(tfar, tnear), nw)))
        low, high, mid = 0.0, r32(1.732), r32(0.0001)
        found, done, first = False, False, True
        delta = int(math.floor(mul(r32(0.15), float(S))))
        while not found or not done:
            passes += 1
            if found:
                done = True
            thresh = mid
            nterm = 0
            is_open = False
            start = end = 0.0
            last = transparent = False
            adj = [0.0] * 4
            step = tnear
            wprev = vmix(wfront, wback, sub(step, nw))
            ndc_step = 0.0
            k_in = k_tt = 0
            cur = [0.0] * 4
            for i in range(num_steps):
                if i == num_steps - 1:
                    last = True
                wpos = vmix(wfront, wback, step)
                if vis and step > lnear and step < lfar:
                    transparent = False
                    x = vol.sample(wpos)
                    if x[0] > -0.5 or last:
                        w = adjust_opacity(x[3], length(vsub(wpos, wprev)))
                        if w <= 0.0:
                            transparent = True
                        if is_open:
                            jp = vmix(wfront, wback, mul(nw, float(k_in)))
                            seg = length(vsub(jp, wfront))
                            ia = div(1.0, cur[3])
                            adj = [mul(cur[0], ia), mul(cur[1], ia), mul(cur[2], ia),
                                   adjust_opacity(cur[3], div(1.0, seg))]
                            d = length([sub(mul(adj[c], adj[3]), mul(x[c], x[3])) for c in range(3)])
                            if d >= thresh:
                                nterm += 1
                                is_open = False
                                end = ndc_step
                                k_in = k_tt = 0
                                if found:
                                    close(start, end, adj)
                        if not is_open and not transparent:
                            is_open = True
                            start = divide_w(matvec(pv, wpos))[2]
                            cur = [0.0] * 4
                        if is_open:
                            t = sub(1.0, cur[3])
                            cur = [fma32(mul(t, x[0]), w, cur[0]), fma32(mul(t, x[1]), w, cur[1]),
                                   fma32(mul(t, x[2]), w, cur[2]), fma32(t, w, cur[3])]
                            k_in += 1
                            if not transparent:
                                k_tt = k_in
                                ndc_step = divide_w(matvec(pv, vmix(wfront, wback, add(step, nw))))[2]
                        if last and is_open:
                            jp = vmix(wfront, wback, mul(nw, float(k_tt)))
                            seg = length(vsub(jp, wfront))
                            ia = div(1.0, cur[3])
                            adj = [mul(cur[0], ia), mul(cur[1], ia), mul(cur[2], ia),
                                   adjust_opacity(cur[3], div(1.0, seg))]
                            nterm += 1
                            is_open = False
                            end = ndc_step
                            k_in = 0
                            if found:
                                close(start, end, adj)
                wprev = wpos
                step = add(step, nw)
            if not done:
                if abs(sub(high, low)) < r32(0.000001):
                    found = True
                    mid = low if nterm == 0 else high
                    continue
                elif nterm > S:
                    low = mid
                elif nterm < S - delta:
                    high = mid
                else:
                    found = True
                    continue
                if first:
                    first = False
                    if nterm < S:
                        found = True
                        continue
                mid = div(add(low, high), 2.0)
    return written, cells, passes


def vdi_image(vol: Volume, cam: dict, W: int, H: int, S: int):
    """Whole sub-VDI in the reference layouts: colour[x][y][i] rgba, depth[x][y][2i(+1)], octree
    counts[z][cy][cx], passes[y][x] (nested lists)."""
    color = [[[[0.0] * 4 for _ in range(S)] for _ in range(H)] for _ in range(W)]
    depth = [[[0.0] * (2 * S) for _ in range(H)] for _ in range(W)]
    octree = [[[0] * (W // 8) for _ in range(H // 8)] for _ in range(S)]
    passes = [[0] * W for _ in range(H)]
    for gx in range(W):
        for gy in range(H):
            segs, cells, p = vdi_pixel(vol, cam, gx, gy, W, H, S)
            for i, (s, e, c) in enumerate(segs[:S]):
                color[gx][gy][i] = list(c)
                depth[gx][gy][2 * i], depth[gx][gy][2 * i + 1] = s, e
            for (cx, cy, z) in cells:
                octree[z][cy][cx] += 1
            passes[gy][gx] = p
    return color, depth, octree, passes


# --------------------------------------------------------------- flatten (accumulateSupseg)
def flatten_pixel(lists, ipv, gx, gy, W, H):
    """lists: per sub-VDI a list of (start, end, (r,g,b,a)) in slot order (zero slots included).
    determineNextSupseg order (VDICompositor.comp:58-91) + accumulateSupseg (VDIGenerator.comp:147-185)."""
    ndc_x = fma32(div(float(gx), float(W)), 2.0, -1.0)
    ndc_y = fma32(div(float(gy), float(H)), 2.0, -1.0)
    front = [0] * len(lists)
    C = [0.0] * 4
    while True:
        low, idx = r32(100000.0), -1
        for j, l in enumerate(lists):
            if front[j] >= len(l):
                continue
            s = l[front[j]][0]
            if s < low and s != 0.0:
                low, idx = s, j
        if idx < 0:
            break
        s, e, c = lists[idx][front[idx]]
        sw = divide_w(matvec(ipv, [ndc_x, ndc_y, s, 1.0]))
        ew = divide_w(matvec(ipv, [ndc_x, ndc_y, e, 1.0]))
        a = adjust_opacity(c[3], length(vsub(sw, ew)))
        t = sub(1.0, C[3])
        C = [fma32(mul(t, c[0]), a, C[0]), fma32(mul(t, c[1]), a, C[1]), fma32(mul(t, c[2]), a, C[2]),
             fma32(t, a, C[3])]
        front[idx] += 1
    return [unorm8(v) for v in C]


# --------------------------------------------------------------- VDICompositor.comp
def composite_pixel(lists, ipv, gx, gy, W, H, S_out):
    """Re-supersegmenting compositor of one pixel (VDICompositor.comp:152-469), written from the
    GLSL.  lists: per sub-VDI [(start, end, (r,g,b,a))] in slot order.  Returns (slots, passes)
    with slots = S_out tuples (start, end, (r,g,b,a))."""
    ndc_x = fma32(div(float(gx), float(W)), 2.0, -1.0)
    ndc_y = fma32(div(float(gy), float(H)), 2.0, -1.0)

    def world(z):
        return divide_w(matvec(ipv, [ndc_x, ndc_y, z, 1.0]))

    def dist(a, b):
        return length(vsub(a, b))

    out = [(0.0, 0.0, (0.0, 0.0, 0.0, 0.0))] * S_out
    num = 0
    low, high = 0.0, r32(1.732)
    mid = div(add(high, low), 2.0)
    found = written = False
    it = 0
    while not found or not written:
        it += 1
        if it > 64:
            break
        if found:
            written = True
        thresh = mid
        nterm = 0
        is_open = False
        s_start = s_end = s_end_tt = 0.0
        cur = [0.0, 0.0, 0.0, 0.0]
        adj = [0.0, 0.0, 0.0, 0.0]
        front = [0] * len(lists)
        complete = False
        while not complete:
            transparent = False
            start = end = 0.0
            colour = [0.0, 0.0, 0.0, 0.0]
            lowd, pid = r32(100000.0), -1
            for j, l in enumerate(lists):
                if front[j] >= len(l):
                    continue
                c = l[front[j]][0]
                if c < lowd and c != 0.0:
                    lowd, pid = c, j
                    start, end, colour = c, l[front[j]][1], list(l[front[j]][2])
            if end == 0.0:
                complete = True
            a_adj = adjust_opacity(colour[3], dist(world(start), world(end)))
            a_adj = gmax(a_adj, r32(0.000001))
            if is_open:
                if start > s_end:
                    transparent = True
                    colour = [0.0, 0.0, 0.0, 0.0]
                    a_adj = 0.0
                    end, start = start, s_end
                sw = world(s_start)
                seg = dist(sw, world(s_end))
                inva = div(1.0, cur[3])
                adj = [mul(cur[0], inva), mul(cur[1], inva), mul(cur[2], inva), adjust_opacity(cur[3], div(1.0, seg))]
                t = sub(1.0, cur[3])
                acc = [fma32(mul(t, colour[k]), a_adj, cur[k]) for k in range(3)] + [fma32(t, a_adj, cur[3])]
                diff = length([sub(mul(adj[k], adj[3]), mul(colour[k], colour[3])) for k in range(3)])
                if diff >= thresh or complete:
                    nterm += 1
                    is_open = False
                    if found:
                        seg_tt = dist(sw, world(s_end_tt))
                        adj[3] = adjust_opacity(cur[3], div(1.0, seg_tt))
                        if num < S_out:
                            out[num] = (s_start, s_end_tt, tuple(adj))
                        num += 1
                else:
                    cur = acc
                    s_end = end
                    if not transparent:
                        s_end_tt = end
            if not is_open and not transparent:
                s_start, s_end, s_end_tt = start, end, end
                cur = [mul(colour[0], a_adj), mul(colour[1], a_adj), mul(colour[2], a_adj), a_adj]
                is_open = True
            if pid != -1 and not transparent:
                front[pid] += 1
        if not written:
            if abs(sub(high, low)) < r32(0.000001):
                found = True
                mid = low if nterm == 0 else high
                continue
            elif nterm > S_out:
                low = mid
            elif nterm < S_out - 3:
                high = mid
            else:
                found = True
                continue
            mid = div(add(low, high), 2.0)
    return out, it


# --------------------------------------------------------------- plain mode
def encode_depth(v):
    enc = [mul(1.0, v), mul(255.0, v), mul(65025.0, v), mul(16581375.0, v)]
    enc = [sub(x, math.floor(x)) for x in enc]
    c = div(1.0, 255.0)
    out = [fma32(-enc[1], c, enc[0]), fma32(-enc[2], c, enc[1]), fma32(-enc[3], c, enc[2]),
           fma32(-enc[3], 0.0, enc[3])]
    return [unorm8(x) for x in out]


def decode_depth(rgba8):
    d = [1.0, div(1.0, 255.0), div(1.0, 65025.0), div(1.0, 16581375.0)]
    v = [div(float(c), 255.0) for c in rgba8]
    t = mul(v[0], d[0])
    for k in range(1, 4):
        t = fma32(v[k], d[k], t)
    return t


def plain_pixel(vol: Volume, cam: dict, gx, gy, dim0, dim1):
    ipv = matmul(cam["inv_view"], cam["inv_proj"])
    nw, fwnw = r32(cam["nw"]), r32(cam.get("fwnw", 0.0))
    _, _, wfront, wback = _ray(ipv, gx, gy, dim0, dim1)
    tnear, tfar = 1.0, 0.0
    n, f = vol.intersect(wfront, wback)
    f = gmin(r32(cam["tmax"]), f)
    vis = False
    if n < f:
        tnear, tfar, vis = gmin(tnear, gmax(0.0, n)), gmax(tfar, f), True
    if not tnear < tfar:
        return [0, 0, 0, 0], [0, 0, 0, 0]
    if fwnw > r32(0.00001):
        ln = lambda x: mul(log2_32(x), r32(0.693147182))  # noqa: E731
        num = int(div(ln(div(fma32(tfar, fwnw, nw), fma32(tnear, fwnw, nw))), ln(add(1.0, fwnw))))
    else:
        num = int(math.trunc(add(div(sub(tfar, tnear), nw), 1.0)))
    step, v = tnear, [0.0] * 4
    for _ in range(num):
        wpos = vmix(wfront, wback, step)
        if vis:
            x = vol.sample(wpos)
            t = sub(1.0, v[3])
            v = [fma32(mul(t, x[0]), x[3], v[0]), fma32(mul(t, x[1]), x[3], v[1]),
                 fma32(mul(t, x[2]), x[3], v[2]), fma32(t, x[3], v[3])]
            if v[3] >= 1.0:
                break
        step = add(step, fma32(step, fwnw, nw))
    return [unorm8(c) for c in v], encode_depth(tnear)


def plain_composite_pixel(colors, depths):
    """colors/depths: per process an rgba8 4-tuple of this pixel (PlainImageCompositor.comp:35-92)."""
    P = len(colors)
    used = [False] * P
    C = [0.0] * 4
    for _ in range(P):
        low, idx, col = r32(200.0), -1, [0.0] * 4
        for j in range(P):
            if used[j]:
                continue
            d = decode_depth(depths[j])
            if d < low and d != 0.0:
                low, idx = d, j
                col = [div(float(c), 255.0) for c in colors[j]]
        t = sub(1.0, C[3])
        C = [fma32(mul(t, col[0]), col[3], C[0]), fma32(mul(t, col[1]), col[3], C[1]),
             fma32(mul(t, col[2]), col[3], C[2]), fma32(t, col[3], C[3])]
        if idx != -1:
            used[idx] = True
    return [unorm8(c) for c in C]
