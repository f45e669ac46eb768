"""A second, independent restatement of render.cpp in pure Python with numpy float32 scalars
(test infrastructure; small frames only -- one Python loop iteration per pixel).

Written separately from oracle/render_oracle.c so that the two can pin each other: the reference
itself cannot be built here (Apple <simd/simd.h>), so "parity" is defined by the restatement, and
agreement of two independent transcriptions guards against transcription slips in either.
Line references are to /root/reference/render-cpp/render.cpp.
"""
from __future__ import annotations

import math
import struct

import numpy as np

from swift3drenderer_amd import scene as scn

F = np.float32
NEAR = F(0.1)                                                   # :90
FOV = F(F(math.pi) / F(5.0))                                    # :91
SCALE = F(NEAR * F(math.tan(float(F(FOV / F(2))))))             # :92
SPEED = F(0.1)                                                  # :94
ROT = F(0.3)                                                    # :95
BG = (30 << 16) | (30 << 8) | 30                                # :96


def v(*a):
    return [F(x) for x in a]


def vadd(a, b):
    return [F(x + y) for x, y in zip(a, b)]


def vsub(a, b):
    return [F(x - y) for x, y in zip(a, b)]


def vmul(a, s):
    return [F(x * s) for x in a]


def smul(s, a):
    return [F(s * x) for x in a]


def dot(a, b):                                                   # simd_dot
    return F(F(F(a[0] * b[0]) + F(a[1] * b[1])) + F(a[2] * b[2]))


def cross(a, b):
    return [F(F(a[1] * b[2]) - F(a[2] * b[1])), F(F(a[2] * b[0]) - F(a[0] * b[2])),
            F(F(a[0] * b[1]) - F(a[1] * b[0]))]


def fnorm(a):                                                    # simd_fast_normalize
    r = F(F(1.0) / F(np.sqrt(dot(a, a))))
    return vmul(a, r)


def act(im, re, x):                                              # simd_act
    t = smul(F(2.0), cross(im, x))
    return vadd(vadd(x, smul(re, t)), cross(im, t))


def u8(f):
    f = float(f)
    if not (abs(f) < 2147483648.0):
        return 0
    return int(f) & 255


def u32(f):
    return int(float(f)) & 0xFFFFFFFF


def npot(i):                                                     # :115-122
    i = (i - 1) & 0xFFFFFFFF
    i |= i >> 1
    i |= i >> 2
    i |= i >> 4
    return (i + 1) & 0xFFFFFFFF


class PyRef:
    def __init__(self, data_path):
        a = scn.read_scene(data_path)
        self.verts = [list(map(F, row)) for row in a.vertices]
        self.vi = [int(x) for x in a.vertex_indices]
        self.ai = [int(x) for x in a.attribute_indices]
        self.attrs = []
        for row in a.attributes:
            b = bytes(row)
            n = list(map(F, struct.unpack_from('<4f', b, 0)))
            disc = struct.unpack_from('<I', b, 32)[0]
            col = list(map(F, struct.unpack_from('<3f', b, 16)))
            idx = struct.unpack_from('<I', b, 16)[0]
            uv = list(map(F, struct.unpack_from('<2f', b, 24)))
            self.attrs.append((n, disc, col, idx, uv))
        self.tex = a.texels
        self.pos = v(0, 0, 0)
        self.ax, self.ay, self.az = v(1, 0, 0), v(0, 1, 0), v(0, 0, 1)
        self.m = [v(1, 0, 0, 0), v(0, 1, 0, 0), v(0, 0, 1, 0)]
        self.mouse = v(0, 0)
        self.factor = F(1)
        self.dbs = 0
        self.init = False

    def camera(self, inp, force):                                # :134-156
        up, down, left, right, mx, my = map(F, inp)
        changed = False
        if left > 0 or right > 0 or up > 0 or down > 0:
            changed = True
            mv = vadd(smul(F(right - left), self.ax), smul(F(down - up), self.az))
            self.pos = vadd(self.pos, smul(SPEED, mv))
        if mx != self.mouse[0] or my != self.mouse[1]:
            changed = True
            d = vadd(vadd(smul(F(self.mouse[0] - mx), self.ax), smul(F(self.mouse[1] - my), self.ay)),
                     smul(F(F(100) / ROT), self.az))
            z = fnorm(d)
            h = fnorm(vadd(self.az, z))
            im, re = cross(self.az, h), dot(self.az, h)
            self.ax = fnorm(act(im, re, self.ax))
            self.ay = fnorm(act(im, re, self.ay))
            self.az = z
            self.mouse = [mx, my]
        if changed or force:
            self.m = [r + [F(-dot(r, self.pos))] for r in (self.ax, self.ay, self.az)]

    def mul(self, p):                                            # simd_mul(float4x3, float4)
        return [F(F(F(F(r[0] * p[0]) + F(r[1] * p[1])) + F(r[2] * p[2])) + F(r[3] * p[3])) for r in self.m]

    def texel(self, base, uvx, uvy, lx_, ly_):                   # :124-132
        lx = npot(u32(max(min(lx_, F(256)), F(1))))
        ly = npot(u32(max(min(ly_, F(256)), F(1))))
        x = (u32(F(F(np.fmod(uvx, F(1))) * F(lx))) + (511 & ~(2 * lx - 1))) & 0xFFFFFFFF
        y = (u32(F(F(np.fmod(uvy, F(1))) * F(ly))) + (511 & ~(2 * ly - 1))) & 0xFFFFFFFF
        off = (x + (y << 9)) & ((1 << 18) - 1)
        rgb = int(self.tex[base + off]) if base + (1 << 18) <= len(self.tex) else 0
        return [F(rgb >> 16), F((rgb >> 8) & 255), F(rgb & 255)]

    def render(self, w, h, inp):                                 # :264-384
        if not self.init:
            self.init = True
            self.camera(inp, True)
        else:
            self.camera(inp, False)
        dbs = (w * h * 4) & 0xFFFFFFFF
        if self.dbs != dbs:
            self.dbs = dbs
            self.factor = F(F(NEAR * F(h)) / F(F(2) * SCALE))
        depth = np.zeros((h, w), dtype=np.float32)
        out = np.full((h, w), BG, dtype=np.uint32)
        sw, sh = F(w), F(h)
        cvs, rvs = [], []
        for p in self.verts:
            c = self.mul(p)
            nz = F(-c[2])
            rvs.append([F(F(F(c[0] * self.factor) / nz) + F(sw / F(2))),
                        F(F(F(F(-c[1]) * self.factor) / nz) + F(sh / F(2))),
                        F(F(F(F(0) * self.factor) / nz) + nz)])
            cvs.append(c)
        cas = [(a[1], a[2], a[3], a[4]) for a in self.attrs]      # (disc, colour, index, uv)
        nrm = [self.mul(a[0]) for a in self.attrs]
        vi, ai = list(self.vi), list(self.ai)
        index = 0
        while index < len(vi) - len(vi) % 3:
            d = [[cvs[vi[index + k]], rvs[vi[index + k]], cas[ai[index + k]], nrm[ai[index + k]]]
                 for k in range(3)]
            vcur = [vi[index + k] for k in range(3)]
            acur = [ai[index + k] for k in range(3)]
            index += 3
            zs = [d[k][1][2] for k in range(3)]
            if max(max(zs[0], zs[1]), zs[2]) <= NEAR:
                continue
            if min(min(zs[0], zs[1]), zs[2]) < NEAR:
                self.clip(d, cvs, rvs, cas, nrm, vi, ai, vcur, acur, sw, sh)
            rv = [d[k][1] for k in range(3)]
            mx = [max(max(rv[0][c], rv[1][c]), rv[2][c]) for c in range(2)]
            if mx[0] < 0 or mx[1] < 0:
                continue
            mn = [min(min(rv[0][c], rv[1][c]), rv[2][c]) for c in range(2)]
            if mn[0] >= sw or mn[1] >= sh:
                continue

            def edge(a, b, cx, cy):
                return F(F(F(cx - a[0]) * F(a[1] - b[1])) + F(F(cy - a[1]) * F(b[0] - a[0])))
            area = edge(rv[0], rv[1], rv[2][0], rv[2][1])
            if area < 10:
                continue
            ooa = F(F(1) / area)
            xmin, xmax = u32(max(F(0), mn[0])), u32(min(F(sw - F(1)), mx[0]))
            ymin, ymax = u32(max(F(0), mn[1])), u32(min(F(sh - F(1)), mx[1]))
            px, py = F(F(xmin) + F(0.5)), F(F(ymin) + F(0.5))
            ws = vmul([edge(rv[1], rv[2], px, py), edge(rv[2], rv[0], px, py), edge(rv[0], rv[1], px, py)], ooa)
            dx = vmul([F(rv[1][1] - rv[2][1]), F(rv[2][1] - rv[0][1]), F(rv[0][1] - rv[1][1])], ooa)
            dy = vmul([F(rv[2][0] - rv[1][0]), F(rv[0][0] - rv[2][0]), F(rv[1][0] - rv[0][0])], ooa)
            rvz = [F(F(1) / rv[k][2]) for k in range(3)]
            cvr = [vmul(d[k][0], rvz[k]) for k in range(3)]
            nr = [vmul(d[k][3], rvz[k]) for k in range(3)]
            disc0 = d[0][2][0]
            if disc0 == 0:
                cc = [vmul(d[k][2][1], rvz[k]) for k in range(3)]
            else:
                base = (d[0][2][2] << 18) & 0xFFFFFFFF
                uv = [vmul(d[k][2][3], rvz[k]) for k in range(3)]
                dz = [dot(rvz, dx), dot(rvz, dy)]
                tpp = [F(F(F(uv[0][0] * dx[0]) + F(uv[1][0] * dx[1])) + F(uv[2][0] * dx[2])),
                       F(F(F(uv[0][1] * dy[0]) + F(uv[1][1] * dy[1])) + F(uv[2][1] * dy[2]))]
            wy = list(ws)
            for y in range(ymin, ymax + 1):
                wv = list(wy)
                for x in range(xmin, xmax + 1):
                    if wv[0] >= 0 and wv[1] >= 0 and wv[2] >= 0:
                        ooz = dot(rvz, wv)
                        if ooz > depth[y, x]:
                            depth[y, x] = ooz
                            ww = [F(q / ooz) for q in wv]
                            P = vadd(vadd(vmul(cvr[0], ww[0]), vmul(cvr[1], ww[1])), vmul(cvr[2], ww[2]))
                            point = [F(-q) for q in fnorm(P)]
                            N = vadd(vadd(vmul(nr[0], ww[0]), vmul(nr[1], ww[1])), vmul(nr[2], ww[2]))
                            normal = fnorm(N)
                            half = fnorm(vadd(point, normal))
                            if disc0 == 0:
                                col = vadd(vadd(vmul(cc[0], ww[0]), vmul(cc[1], ww[1])), vmul(cc[2], ww[2]))
                            else:
                                mp = [F(F(F(uv[0][c] * ww[0]) + F(uv[1][c] * ww[1])) + F(uv[2][c] * ww[2]))
                                      for c in range(2)]
                                lv = [F(ooz / F(abs(F(tpp[c] - F(mp[c] * dz[c]))))) for c in range(2)]
                                col = self.texel(base, mp[0], mp[1], lv[0], lv[1])
                            s = dot(half, normal)
                            out[y, x] = (u8(F(s * col[0])) << 16) | (u8(F(s * col[1])) << 8) | u8(F(s * col[2]))
                    wv = vadd(wv, dx)
                wy = vadd(wy, dy)
        return out

    def clip(self, d, cvs, rvs, cas, nrm, vi, ai, vcur, acur, sw, sh):   # :212-262
        new = [None] * 3
        cur = nxt = pre = 0
        newtri = False
        for i in range(3):
            j = (i + 1) % 3
            if (d[i][1][2] > NEAR) == (d[j][1][2] > NEAR):
                cur, nxt, pre = i, j, (i + 2) % 3
                newtri = d[i][1][2] > NEAR
            else:
                a = F(F(NEAR - d[i][1][2]) / F(d[j][1][2] - d[i][1][2]))
                oma = F(F(1) - a)
                cv = vadd(vmul(d[i][0], oma), vmul(d[j][0], a))
                rv = [F(F(F(cv[0] * self.factor) / NEAR) + F(sw / F(2))),
                      F(F(F(F(-cv[1]) * self.factor) / NEAR) + F(sh / F(2))),
                      F(F(F(F(0) * self.factor) / NEAR) + NEAR)]
                disc = d[0][2][0]
                if disc == 0:
                    ca = (0, vadd(vmul(d[i][2][1], oma), vmul(d[j][2][1], a)), 0, v(0, 0))
                else:
                    ca = (disc, v(0, 0, 0), d[i][2][2], vadd(vmul(d[i][2][3], oma), vmul(d[j][2][3], a)))
                n = vadd(vmul(d[i][3], oma), vmul(d[j][3], a))
                new[i] = [cv, rv, ca, n]
        if newtri:
            d[pre] = new[nxt]
            vc, ac = len(cvs), len(cas)
            cvs += [new[nxt][0], new[pre][0]]
            rvs += [new[nxt][1], new[pre][1]]
            cas += [new[nxt][2], new[pre][2]]
            nrm += [new[nxt][3], new[pre][3]]
            # appended at the end of the index arrays: the frame loop reaches it after the originals
            vi += [vcur[cur], vc, vc + 1]
            ai += [acur[cur], ac, ac + 1]
        else:
            d[cur] = new[pre]
            d[nxt] = new[nxt]


def render_pose(data_path, script, w, h):
    r = PyRef(data_path)
    out = None
    for t in script:
        out = r.render(w, h, t)
    return out
