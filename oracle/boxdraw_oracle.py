"""CPU restatement of the box drawing in the reference's step-1 / step-2 prompts — TEST
INFRASTRUCTURE ONLY (tests and ``smoke()`` compare the HIP kernels of csrc/boxdraw.hip with it;
the product package never imports it).

The reference draws boxes into the training image with detectron2's ``Visualizer``
(cullavo/arch_cullavo.py:149-153 step 1, :441-448 step 2 with boxes):

    vis = Visualizer(img_hwc); vis._default_font_size = 16
    out = vis.overlay_instances(boxes=..., assigned_colors=colors, alpha=1).get_image()

detectron2 is not in /root/reference nor importable here (pinned version unknown; its
``utils/visualizer.py`` has been stable since v0.1). What that code does, restated from the
published source:

* ``VisImage`` (visualizer.py ``VisImage._setup_figure`` / ``reset_image`` / ``get_image``): a
  matplotlib ``Figure(frameon=False)`` of (W + 1e-2) x (H + 1e-2) pixels at the default dpi
  (100), one axes over the whole figure with the axis off, ``ax.imshow(img, extent=(0, W, H, 0),
  interpolation="nearest")``, rendered by ``FigureCanvasAgg``; ``get_image`` returns the RGB of
  the canvas buffer.
* ``overlay_instances(boxes, assigned_colors)``: boxes as a float array, drawn largest area first
  (``np.argsort(-areas)``), each with ``draw_box(box, edge_color=color)`` whose defaults are
  alpha 0.5 and line style "-"; ``draw_box`` adds ``Rectangle((x0, y0), x1 - x0, y1 - y0,
  fill=False, linewidth=max(font_size / 4, 1) * scale)`` -> 4 pt at font size 16.

What matplotlib 3.10.8 (installed here; its vendored Agg 2.4) then does to the pixels — restated
from Agg's and matplotlib's C++ sources and checked bit-exactly against the real renderer by
tests/golden/make_golden_boxes.py (fixtures in tests/golden/boxdraw.npz):

* ``visimage_maps`` — imshow "nearest": the (W+0.01)-wide axes round up to a (W+1) x (H+1)
  resample buffer (image.py ``_make_image``), sampled by Agg's ``span_image_filter_rgba_nn``
  through ``span_interpolator_linear`` (24.8 fixed point, ``dda2_line_interpolator`` along a
  row); the buffer is blended bottom-left aligned, so its top row falls off the canvas. Net
  effect: canvas pixel (r, c) = source (rows[r], cols[c]) with rows/cols below.
* ``stroke_outline`` — the Rectangle path transformed to canvas pixels (y down; imshow's equal
  aspect shrinks and centres the axes box, see ``_rect_pixels``), snapped by ``PathSnapper``
  (all segments axis-aligned: vertex -> floor(v + 0.5) + (0.5 if round(width_px) is odd else
  0)), cut by ``PathClipper`` to (-1, -1, W + 1, H + 1) (``agg::clip_line_segment`` per
  segment; a clipped path is no longer closed, each visible run becomes an open subpath), then
  ``vcgen_stroke`` / ``math_stroke`` with width 4 pt =
  5.5556 px, miter joins (limit = width in px), inner miter joins (limit 1.01, reverting to
  bevel), butt caps; consecutive duplicate vertices dropped (``vertex_dist_epsilon`` 1e-14), a
  closed path with fewer than 3 vertices stroked as an open line.
* ``rasterize`` — ``rasterizer_cells_aa::line`` / ``render_hline`` (24.8 fixed point, exact
  integer cell cover/area), ``sweep_scanline`` with ``calculate_alpha`` ((cover << 9) - area)
  >> 9, |.|, clamp 255 (non-zero rule).
* ``blend`` — ``renderer_scanline_aa_solid`` over ``pixfmt_rgba32_plain`` with matplotlib's
  ``fixed_blender_rgba_plain``: alpha = mult_cover(a8, cover), a8 = uround(0.5 * 255) = 128;
  the canvas is opaque after imshow.

Known limit: matplotlib composes the data -> pixel transform from several affine matrices and
bounding boxes; ``_rect_pixels`` evaluates the same mapping in one expression, which can differ
from it in the last ulp, i.e. only where a vertex lands exactly on a snapping or clipping
boundary (not seen in the fixtures).
"""
from __future__ import annotations

import math

import numpy as np

DPI = 100.0
VERTEX_DIST_EPS = 1e-14
INTERSECTION_EPS = 1e-30
COLOR_RGB = {  # matplotlib named colours (CSS4) for the reference's color_list (cullavo/utils/utils.py:14-33)
    "white": (255, 255, 255), "red": (255, 0, 0), "orange": (255, 165, 0), "coral": (255, 127, 80),
    "yellow": (255, 255, 0), "green": (0, 128, 0), "blue": (0, 0, 255), "navy": (0, 0, 128),
    "gold": (255, 215, 0), "pink": (255, 192, 203), "purple": (128, 0, 128), "brown": (165, 42, 42),
    "violet": (238, 130, 238), "olive": (128, 128, 0), "lime": (0, 255, 0), "cyan": (0, 255, 255),
    "magenta": (255, 0, 255), "silver": (192, 192, 192), "gray": (128, 128, 128), "black": (0, 0, 0),
}


def iround(v: float) -> int:
    """agg::iround: int(v -/+ 0.5) truncated toward zero"""
    return int(v - 0.5) if v < 0.0 else int(v + 0.5)


def _cdiv(p: int, d: int):
    """C's p / d and p % d (truncation toward zero)"""
    q = abs(p) // abs(d)
    if (p < 0) != (d < 0):
        q = -q
    return q, p - q * d


# ---- VisImage geometry: matplotlib's figure / axes / image transforms --------------------------------
def _dot(b, a):
    """np.dot(B, A) of two [[sx, 0, tx], [0, sy, ty], [0, 0, 1]] matrices stored (sx, tx, sy, ty)"""
    return (b[0] * a[0], b[0] * a[1] + b[1], b[2] * a[2], b[2] * a[3] + b[3])


def _apply(m, x, y):
    return m[0] * x + m[1], m[2] * y + m[3]


def axes_transform(H: int, W: int, dpi: float = DPI):
    """ax.transData of VisImage as (sx, tx, sy, ty) (display y up) and the axes bbox.

    Figure (W + 1e-2) x (H + 1e-2) px; imshow sets aspect "equal", so Axes.apply_aspect
    shrinks the [0, 0, 1, 1] position with Bbox.shrunk_to_aspect(box_aspect = H / W,
    fig_aspect = fig height / width in px) and re-anchors it at "C" (Bbox.anchored); transData =
    BboxTransformTo(ax.bbox) . BboxTransformFrom(viewLim = (0, H) -> (W, 0)). Same operations in
    the same order as matplotlib 3.10 (transforms.py), so the doubles are bit-identical."""
    w_in, h_in = (W + 1e-2) / dpi, (H + 1e-2) / dpi
    fw, fh = w_in * dpi, h_in * dpi
    fig_aspect = fh / fw
    box_aspect = 1.0 * (abs(0.0 - H) / abs(W - 0.0))
    hh = 1.0 * box_aspect / fig_aspect
    if hh <= 1.0:
        ww = 1.0
    else:
        ww = 1.0 * fig_aspect / box_aspect
        hh = 1.0
    ox = (0.0 + 0.5 * (1.0 - ww)) - 0.0
    oy = (0.0 + 0.5 * (1.0 - hh)) - 0.0
    sub = (fw - 0.0, 0.0, fh - 0.0, 0.0)  # transSubfigure = BboxTransformTo(fig.bbox)
    ax0, ay0 = _apply(sub, 0.0 + ox, 0.0 + oy)
    ax1, ay1 = _apply(sub, ww + ox, hh + oy)
    inw, inh = W - 0.0, 0.0 - H
    xs, ys = 1.0 / inw, 1.0 / inh
    frm = (xs, -0.0 * xs, ys, -float(H) * ys)
    to = (ax1 - ax0, ax0, ay1 - ay0, ay0)
    return _dot(to, frm), (ax0, ay0, ax1, ay1)


def image_matrix(H: int, W: int):
    """the source -> resample-buffer affine of imshow (image.py _ImageBase._make_image, origin
    "upper", extent (0, W, H, 0), magnification 1) and the buffer shape (rows, cols)"""
    td, (ax0, ay0, ax1, ay1) = axes_transform(H, W)
    a1 = (1.0, 0.0, -1.0, (0.0 - H) * -1.0)                 # translate(0, -H).scale(1, -1)
    a2 = (W / W, 0.0 * (W / W) + 0.0, (0.0 - H) / H, 0.0 + float(H))  # scale(...).translate(0, H)
    t = _dot(_dot(td, a2), a1)
    p0, p1 = _apply(td, 0.0, float(H)), _apply(td, float(W), 0.0)
    cx0 = max(min(p0[0], p1[0]), min(ax0, ax1))
    cx1 = min(max(p0[0], p1[0]), max(ax0, ax1))
    cy0 = max(min(p0[1], p1[1]), min(ay0, ay1))
    cy1 = min(max(p0[1], p1[1]), max(ay0, ay1))
    t = _dot((1.0, -cx0 * 1.0, 1.0, -cy0 * 1.0), t)
    owb, ohb = (cx1 - cx0) * 1.0, (cy1 - cy0) * 1.0
    if owb % 1.0 != 0.0 or ohb % 1.0 != 0.0:
        ow, oh = math.ceil(owb), math.ceil(ohb)
        t = _dot((1.0 + (ow - owb) / owb, 0.0, 1.0 + (oh - ohb) / ohb, 0.0), t)
    else:
        ow, oh = int(owb), int(ohb)
    return t, (oh, ow)


def _dda2(y1: int, y2: int, count: int):
    """agg::dda2_line_interpolator(y1, y2, count): the count values it yields"""
    cnt = count if count > 0 else 1
    lft, rem = _cdiv(y2 - y1, cnt)
    mod = rem
    y = y1
    if mod <= 0:
        mod += count
        rem += count
        lft -= 1
    mod -= count
    out = []
    for _ in range(count):
        out.append(y)
        mod += rem
        y += lft
        if mod > 0:
            mod -= cnt
            y += 1
    return out


def visimage_maps(H: int, W: int):
    """source row / column of every canvas pixel of VisImage(img).get_image() with no drawing.

    _image.resample with "nearest": agg::trans_affine::invert of image_matrix, then per output
    scanline span_interpolator_linear::begin(0.5, y + 0.5, buffer width) (24.8 fixed point,
    dda2 along the row) and span_image_filter_rgba_nn (source = coordinate >> 8). The buffer
    (H + 1 rows) is blended at canvas row int(H - (cy0 + H + 1)) = -1: canvas row r shows buffer
    row r + 1 from the top, i.e. buffer scanline (rows - 2 - r) counted from the bottom."""
    (sx, tx, sy, ty), (oh, ow) = image_matrix(H, W)
    d = 1.0 / (sx * sy - 0.0 * 0.0)
    ishx, ishy = -0.0 * d, -0.0 * d
    isx, isy = sy * d, sx * d
    itx = -tx * isx - ty * ishx
    ity = -tx * ishy - ty * isy

    def tr(x, y):
        return x * isx + y * ishx + itx, x * ishy + y * isy + ity
    xs = _dda2(iround(tr(0.5, 0.5)[0] * 256), iround(tr(0.5 + ow, 0.5)[0] * 256), ow)
    cols = np.array([x >> 8 for x in xs[:W]], np.int64)
    rows = np.array([iround(tr(0.5, (oh - 2 - r) + 0.5)[1] * 256) >> 8 for r in range(H)], np.int64)
    return rows, cols


# ---- Rectangle path -> canvas pixels, PathClipper, PathSnapper ---------------------------------
def _rect_pixels(box, H: int, W: int):
    """the Rectangle's 4 vertices in canvas pixels (y down), before clipping and snapping.

    draw_box builds Rectangle((x0, y0), x1 - x0, y1 - y0) from the float32 box, so the far
    corner is float32(x0 + float32(x1 - x0)); the patch transform is BboxTransformTo(its bbox)
    (the rotation part is the identity), composed with transData (np.dot), converted to
    agg::trans_affine and flipped by RendererAgg::draw_path (scaling(1, -1), translation(0, H))."""
    x0, y0, x1, y1 = (np.float32(v) for v in box)
    x1 = np.float32(x0 + np.float32(x1 - x0))
    y1 = np.float32(y0 + np.float32(y1 - y0))
    td, _ = axes_transform(H, W)
    sx, tx, sy, ty = _dot(td, (float(x1) - float(x0), float(x0), float(y1) - float(y0), float(y0)))
    ty = -ty + float(H)
    sy = -sy
    X0, X1 = tx, sx + tx
    Y0, Y1 = ty, sy + ty
    return [(X0, Y0), (X1, Y0), (X1, Y1), (X0, Y1)]


def _clip_flags(x, y, r):
    return int(x > r[2]) | (int(y > r[3]) << 1) | (int(x < r[0]) << 2) | (int(y < r[1]) << 3)


def _clip_segment(x1, y1, x2, y2, r):
    """agg::clip_line_segment: (moved, x1, y1, x2, y2); moved >= 4 fully clipped"""
    f1, f2 = _clip_flags(x1, y1, r), _clip_flags(x2, y2, r)
    if (f1 | f2) == 0:
        return 0, x1, y1, x2, y2
    if (f1 & 5) and (f1 & 5) == (f2 & 5):
        return 4, x1, y1, x2, y2
    if (f1 & 10) and (f1 & 10) == (f2 & 10):
        return 4, x1, y1, x2, y2
    tx1, ty1, tx2, ty2 = x1, y1, x2, y2
    ret = 0

    def move(px_, py_, flags):
        if flags & 5:
            if tx1 == tx2:
                return None
            bound = r[0] if flags & 4 else r[2]
            py_ = (bound - tx1) * (ty2 - ty1) / (tx2 - tx1) + ty1
            px_ = bound
        fy = (int(py_ > r[3]) << 1) | (int(py_ < r[1]) << 3)
        if fy & 10:
            if ty1 == ty2:
                return None
            bound = r[1] if fy & 8 else r[3]
            px_ = (bound - ty1) * (tx2 - tx1) / (ty2 - ty1) + tx1
            py_ = bound
        return px_, py_
    if f1:
        m = move(x1, y1, f1)
        if m is None:
            return 4, x1, y1, x2, y2
        x1, y1 = m
        if x1 == x2 and y1 == y2:
            return 4, x1, y1, x2, y2
        ret |= 1
    if f2:
        m = move(x2, y2, f2)
        if m is None:
            return 4, x1, y1, x2, y2
        x2, y2 = m
        if x1 == x2 and y1 == y2:
            return 4, x1, y1, x2, y2
        ret |= 2
    return ret, x1, y1, x2, y2


def clip_rect_path(pts, H: int, W: int):
    """matplotlib PathClipper (path_converters.h) on MOVETO v0, LINETO v1..v3, CLOSEPOLY with the
    clip rectangle (-1, -1, W + 1, H + 1): [(vertices, closed)] subpaths"""
    r = (-1.0, -1.0, W + 1.0, H + 1.0)
    subs, cur = [], None
    moveto, was_clipped = True, False
    segs = [(pts[k], pts[(k + 1) % 4], k == 3) for k in range(4)]
    for (a, b, closing) in segs:
        moved, x0, y0, x1, y1 = _clip_segment(a[0], a[1], b[0], b[1], r)
        was_clipped = was_clipped or moved != 0
        if moved < 4:
            if (moved & 1) or moveto:
                cur = [(x0, y0), (x1, y1)]
                subs.append([cur, False])
            else:
                cur.append((x1, y1))
            if closing and not was_clipped:
                subs[-1][1] = True
            moveto = False
    return [(v, c) for v, c in subs]


def snap(pts, width_px: float):
    """PathSnapper: every segment axis-aligned -> floor(v + 0.5) + (0.5 if round(width) is odd)"""
    sv = 0.5 if iround(width_px) % 2 else 0.0
    return [(math.floor(x + 0.5) + sv, math.floor(y + 0.5) + sv) for x, y in pts]


def _dist(a, b):
    return math.sqrt((b[0] - a[0]) ** 2 + (b[1] - a[1]) ** 2)


def _dedup(pts, closed: bool):
    """agg::vertex_sequence<vertex_dist>::add + close(closed)"""
    seq = []
    for p in pts:
        if len(seq) > 1 and not _dist(seq[-2], seq[-1]) > VERTEX_DIST_EPS:
            seq.pop()
        seq.append(p)
    while len(seq) > 1 and not _dist(seq[-2], seq[-1]) > VERTEX_DIST_EPS:
        t = seq.pop()
        seq[-1] = t
    if closed:
        while len(seq) > 1 and not _dist(seq[-1], seq[0]) > VERTEX_DIST_EPS:
            seq.pop()
    return seq


def _cross(x1, y1, x2, y2, x, y):
    return (x - x2) * (y2 - y1) - (y - y2) * (x2 - x1)


def _intersection(ax, ay, bx, by, cx, cy, dx, dy):
    num = (ay - cy) * (dx - cx) - (ax - cx) * (dy - cy)
    den = (bx - ax) * (dy - cy) - (by - ay) * (dx - cx)
    if abs(den) < INTERSECTION_EPS:
        return None
    r = num / den
    return ax + r * (bx - ax), ay + r * (by - ay)


def _miter(out, v0, v1, v2, dx1, dy1, dx2, dy2, revert, mlimit, hw):
    """agg::math_stroke::calc_miter for miter_join (outer) / miter_join_revert (inner)"""
    lim = hw * mlimit
    exceeded = True
    p = _intersection(v0[0] + dx1, v0[1] - dy1, v1[0] + dx1, v1[1] - dy1,
                      v1[0] + dx2, v1[1] - dy2, v2[0] + dx2, v2[1] - dy2)
    if p is not None:
        if _dist(v1, p) <= lim:
            out.append(p)
            exceeded = False
    else:
        x2, y2 = v1[0] + dx1, v1[1] - dy1
        if (_cross(v0[0], v0[1], v1[0], v1[1], x2, y2) < 0.0) == (_cross(v1[0], v1[1], v2[0], v2[1], x2, y2) < 0.0):
            out.append((v1[0] + dx1, v1[1] - dy1))
            exceeded = False
    if exceeded:
        if revert or p is None:
            # miter_join_revert: bevel. (The outer miter of an axis-aligned rectangle never
            # exceeds its limit: sqrt(2) < width in px.)
            out.append((v1[0] + dx1, v1[1] - dy1))
            out.append((v1[0] + dx2, v1[1] - dy2))
        else:
            raise AssertionError("outer miter beyond its limit")


def _join(out, v0, v1, v2, len1, len2, hw, miter_limit):
    """agg::math_stroke::calc_join (line_join miter, inner_join inner_miter)"""
    dx1 = hw * (v1[1] - v0[1]) / len1
    dy1 = hw * (v1[0] - v0[0]) / len1
    dx2 = hw * (v2[1] - v1[1]) / len2
    dy2 = hw * (v2[0] - v1[0]) / len2
    cp = _cross(v0[0], v0[1], v1[0], v1[1], v2[0], v2[1])
    if cp > VERTEX_DIST_EPS:  # inner join (width > 0)
        limit = max(min(len1, len2) / hw, 1.01)
        _miter(out, v0, v1, v2, dx1, dy1, dx2, dy2, True, limit, hw)
    else:
        _miter(out, v0, v1, v2, dx1, dy1, dx2, dy2, False, miter_limit, hw)


def _cap(out, v0, v1, length, hw):
    """agg::math_stroke::calc_cap, butt cap"""
    dx1 = (v1[1] - v0[1]) / length * hw
    dy1 = (v1[0] - v0[0]) / length * hw
    out.append((v0[0] - dx1, v0[1] + dy1))
    out.append((v0[0] + dx1, v0[1] - dy1))


def _stroke(seq, closed: bool, hw: float, width_px: float):
    """agg::vcgen_stroke over one subpath -> polygons"""
    n = len(seq)
    if closed and n < 3:
        closed = False
    if n < 2:
        return []
    if closed:
        dist = [_dist(seq[i], seq[(i + 1) % n]) for i in range(n)]
        out1, out2 = [], []
        for i in range(n):  # outline1: joins in path order
            _join(out1, seq[i - 1], seq[i], seq[(i + 1) % n], dist[i - 1], dist[i], hw, width_px)
        for i in range(n - 1, -1, -1):  # outline2: reversed
            _join(out2, seq[(i + 1) % n], seq[i], seq[i - 1], dist[i], dist[i - 1], hw, width_px)
        return [out1, out2]
    dist = [_dist(seq[i], seq[i + 1]) for i in range(n - 1)]
    poly = []
    _cap(poly, seq[0], seq[1], dist[0], hw)
    for i in range(1, n - 1):
        _join(poly, seq[i - 1], seq[i], seq[i + 1], dist[i - 1], dist[i], hw, width_px)
    _cap(poly, seq[n - 1], seq[n - 2], dist[n - 2], hw)
    for i in range(n - 2, 0, -1):
        _join(poly, seq[i + 1], seq[i], seq[i - 1], dist[i], dist[i - 1], hw, width_px)
    return [poly]


def stroke_outline(box, H: int, W: int, width_px: float):
    """contours (lists of (x, y) canvas pixels, y down) of the stroked, clipped Rectangle"""
    hw = width_px * 0.5
    polys = []
    for verts, closed in clip_rect_path(_rect_pixels(box, H, W), H, W):
        polys += _stroke(_dedup(snap(verts, width_px), closed), closed, hw, width_px)
    return polys


# ---- Agg scanline rasterizer (cells) ----------------------------------------------------------------
class _Cells:
    def __init__(self):
        self.cells = {}

    def add(self, ex, ey, cover, area):
        c = self.cells.setdefault((ey, ex), [0, 0])
        c[0] += cover
        c[1] += area

    def hline(self, ey, x1, y1, x2, y2):
        ex1, ex2 = x1 >> 8, x2 >> 8
        fx1, fx2 = x1 & 255, x2 & 255
        if y1 == y2:
            return
        if ex1 == ex2:
            d = y2 - y1
            self.add(ex1, ey, d, (fx1 + fx2) * d)
            return
        p = (256 - fx1) * (y2 - y1)
        first, incr, dx = 256, 1, x2 - x1
        if dx < 0:
            p = fx1 * (y2 - y1)
            first, incr, dx = 0, -1, -dx
        delta, mod = _cdiv(p, dx)
        if mod < 0:
            delta -= 1
            mod += dx
        self.add(ex1, ey, delta, (fx1 + first) * delta)
        ex1 += incr
        y1 += delta
        if ex1 != ex2:
            lift, rem = _cdiv(256 * (y2 - y1 + delta), dx)
            if rem < 0:
                lift -= 1
                rem += dx
            mod -= dx
            while ex1 != ex2:
                delta = lift
                mod += rem
                if mod >= 0:
                    mod -= dx
                    delta += 1
                self.add(ex1, ey, delta, 256 * delta)
                y1 += delta
                ex1 += incr
        delta = y2 - y1
        self.add(ex2, ey, delta, (fx2 + 256 - first) * delta)

    def line(self, x1, y1, x2, y2):
        dx, dy = x2 - x1, y2 - y1
        ey1, ey2 = y1 >> 8, y2 >> 8
        fy1, fy2 = y1 & 255, y2 & 255
        if ey1 == ey2:
            self.hline(ey1, x1, fy1, x2, fy2)
            return
        incr = 1
        if dx == 0:
            ex = x1 >> 8
            two_fx = (x1 - (ex << 8)) << 1
            first = 256
            if dy < 0:
                first, incr = 0, -1
            delta = first - fy1
            self.add(ex, ey1, delta, two_fx * delta)
            ey1 += incr
            delta = first + first - 256
            while ey1 != ey2:
                self.add(ex, ey1, delta, two_fx * delta)
                ey1 += incr
            delta = fy2 - 256 + first
            self.add(ex, ey1, delta, two_fx * delta)
            return
        p = (256 - fy1) * dx
        first = 256
        if dy < 0:
            p = fy1 * dx
            first, incr, dy = 0, -1, -dy
        delta, mod = _cdiv(p, dy)
        if mod < 0:
            delta -= 1
            mod += dy
        x_from = x1 + delta
        self.hline(ey1, x1, fy1, x_from, first)
        ey1 += incr
        if ey1 != ey2:
            lift, rem = _cdiv(256 * dx, dy)
            if rem < 0:
                lift -= 1
                rem += dy
            mod -= dy
            while ey1 != ey2:
                delta = lift
                mod += rem
                if mod >= 0:
                    mod -= dy
                    delta += 1
                x_to = x_from + delta
                self.hline(ey1, x_from, 256 - first, x_to, first)
                x_from = x_to
                ey1 += incr
        self.hline(ey1, x_from, 256 - first, x2, fy2)


def rasterize(contours, H: int, W: int) -> np.ndarray:
    """coverage [H, W] (0..255) of the contours, closed, non-zero rule"""
    cells = _Cells()
    for poly in contours:
        pts = [(iround(x * 256), iround(y * 256)) for x, y in poly]
        for k in range(len(pts)):
            cells.line(*pts[k], *pts[(k + 1) % len(pts)])
    cov = np.zeros((H, W), np.int64)
    rows = {}
    for (ey, ex), (c, a) in cells.cells.items():
        if 0 <= ey < H:
            rows.setdefault(ey, []).append((ex, c, a))
    for ey, cl in rows.items():
        cover_at = np.zeros(W + 1, np.int64)  # [0]: cells left of the canvas (rasterizer clip)
        area_at = np.zeros(W, np.int64)
        for ex, c, a in cl:
            if ex < 0:
                cover_at[0] += c
            elif ex < W:
                cover_at[ex + 1] += c
                area_at[ex] += a
        run = np.cumsum(cover_at)[1:]  # cover of every cell <= x
        val = (run << 9) - area_at
        cov[ey] = np.minimum(np.abs(val >> 9), 255)
    return cov


def mult_cover(a, cover):
    t = a * cover + 128
    return ((t >> 8) + t) >> 8


def blend(canvas: np.ndarray, cover: np.ndarray, rgb, a8: int = 128) -> np.ndarray:
    """fixed_blender_rgba_plain::blend_pix on an opaque canvas (HWC uint8)"""
    al = mult_cover(a8, cover.astype(np.int64))
    p = canvas.astype(np.int64)
    r = p * 255
    A = ((al + 255) << 8) - al * 255
    c = np.asarray(rgb, np.int64)
    new = (((c[None, None, :] << 8) - r) * al[..., None] + (r << 8)) // np.maximum(A, 1)[..., None]
    if a8 == 255:  # blend_solid_hspan: an opaque colour at full cover is copied
        new = np.where((cover >= 255)[..., None], c[None, None, :], new)
    return np.where((al > 0)[..., None], new, p).astype(np.uint8)


def draw_order(boxes) -> list:
    """overlay_instances: largest area first, np.argsort(-areas) on the float32 boxes"""
    b = np.asarray(boxes, np.float32).reshape(-1, 4)
    areas = np.prod(b[:, 2:] - b[:, :2], axis=1)
    return np.argsort(-areas).tolist()


def overlay_boxes(img_hwc: np.ndarray, boxes, colors, font_size: float = 16.0, alpha: float = 0.5) -> np.ndarray:
    """Visualizer(img); _default_font_size = font_size; overlay_instances(boxes=boxes,
    assigned_colors=colors).get_image() — img uint8 [H, W, 3], boxes [n, 4] x0 y0 x1 y1 in
    pixels, colors names of COLOR_RGB or (r, g, b)"""
    img = np.asarray(img_hwc, np.uint8)
    H, W = img.shape[:2]
    rows, cols = visimage_maps(H, W)
    canvas = img[rows][:, cols]
    width_px = max(font_size / 4.0, 1.0) * DPI / 72.0
    a8 = iround(alpha * 255)
    for i in draw_order(boxes) if len(boxes) else []:
        rgb = COLOR_RGB[colors[i]] if isinstance(colors[i], str) else colors[i]
        cov = rasterize(stroke_outline(np.asarray(boxes, np.float32).reshape(-1, 4)[i], H, W, width_px), H, W)
        canvas = blend(canvas, cov, rgb, a8)
    return canvas
