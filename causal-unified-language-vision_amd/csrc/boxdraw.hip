// Box drawing of the reference's step-1 / step-2 prompts (cullavo/arch_cullavo.py:149-153 and
// :441-448): detectron2's Visualizer(img).overlay_instances(boxes, assigned_colors).get_image(),
// i.e. a matplotlib Agg canvas showing the image with one stroked Rectangle per box, restated so
// the pixels are bit-identical. oracle/boxdraw_oracle.py is the CPU restatement (pinned to
// matplotlib 3.10.8's renderer by tests/golden/make_golden_boxes.py); the function names below
// follow it.
//
// Two launches per image size:
//  1. box_outline_k — one thread per box: Rectangle -> canvas pixels (transData from
//     cullavo_visimage_geometry, the f32 corner arithmetic of the Rectangle patch, Agg's y flip),
//     PathClipper (each segment cut to (-1, -1, W+1, H+1); a clipped ring is no longer closed),
//     PathSnapper, vcgen_stroke (miter joins, inner-miter joins reverting to bevel, butt caps)
//     -> closed contours in Agg's 24.8 fixed point, plus their cell extent.
//  2. box_rows_k — one wave per (image, canvas row): the row is gathered into LDS (imshow
//     "nearest": src row rows[r], columns cols[x]); then for each box in draw order the lanes
//     turn the contour edges that cross the row into Agg cells (rasterizer_cells_aa::line /
//     render_hline: exact integer cover and area) in LDS, and each lane takes pixels:
//     coverage = min(|((sum of cover of cells <= x) << 9) - area(x)| >> 9, 255)
//     (sweep_scanline, non-zero rule), blended by fixed_blender_rgba_plain with
//     alpha = mult_cover(a8, coverage). The row leaves LDS once, coalesced.
// Every double operation is written in the order of the matplotlib / Agg code it restates, with
// contraction off, so vertices land on the same side of every rounding and snapping boundary.
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr int kMaxV = 64;       // stroke vertices per box (<= 4 subpaths x 16)
constexpr int kMaxC = 8;        // contours per box
constexpr int kMaxSub = 4;      // clipped subpaths of one rectangle (one per segment at most)
constexpr int kMaxCells = 512;  // Agg cells of one box in one row
constexpr int kMaxW = 8192;     // LDS row buffer: 3 x kMaxW bytes

struct BoxOutline {
  int32_t n_contours, n_vert;
  int32_t ex0, ex1, ey0, ey1;  // cell extent (inclusive); ey0 > ey1 when nothing is drawn
  int32_t start[kMaxC + 1];    // contour k = vertices [start[k], start[k + 1])
  int32_t x[kMaxV], y[kMaxV];  // 24.8 fixed point, canvas pixels, y down
};

struct P {
  double x, y;
};

__host__ __device__ inline int agg_iround(double v) { return (int)((v < 0.0) ? v - 0.5 : v + 0.5); }

// ---- PathClipper (matplotlib path_converters.h) with agg::clip_line_segment ------------------------
DEV int clip_flags(double x, double y, const double* r) {
  return (int)(x > r[2]) | ((int)(y > r[3]) << 1) | ((int)(x < r[0]) << 2) | ((int)(y < r[1]) << 3);
}

DEV bool clip_move_point(double x1, double y1, double x2, double y2, const double* r, double* x, double* y,
                         int flags) {
  if (flags & 5) {
    if (x1 == x2) return false;
    const double bound = (flags & 4) ? r[0] : r[2];
    *y = (bound - x1) * (y2 - y1) / (x2 - x1) + y1;
    *x = bound;
  }
  const int fy = ((int)(*y > r[3]) << 1) | ((int)(*y < r[1]) << 3);
  if (fy & 10) {
    if (y1 == y2) return false;
    const double bound = (fy & 8) ? r[1] : r[3];
    *x = (bound - y1) * (x2 - x1) / (y2 - y1) + x1;
    *y = bound;
  }
  return true;
}

// returns moved: 0 visible, bit 0 first point moved, bit 1 second moved, >= 4 fully clipped
DEV int clip_line_segment(double* x1, double* y1, double* x2, double* y2, const double* r) {
  const int f1 = clip_flags(*x1, *y1, r), f2 = clip_flags(*x2, *y2, r);
  if ((f2 | f1) == 0) return 0;
  if ((f1 & 5) != 0 && (f1 & 5) == (f2 & 5)) return 4;
  if ((f1 & 10) != 0 && (f1 & 10) == (f2 & 10)) return 4;
  const double tx1 = *x1, ty1 = *y1, tx2 = *x2, ty2 = *y2;
  int ret = 0;
  if (f1) {
    if (!clip_move_point(tx1, ty1, tx2, ty2, r, x1, y1, f1)) return 4;
    if (*x1 == *x2 && *y1 == *y2) return 4;
    ret |= 1;
  }
  if (f2) {
    if (!clip_move_point(tx1, ty1, tx2, ty2, r, x2, y2, f2)) return 4;
    if (*x1 == *x2 && *y1 == *y2) return 4;
    ret |= 2;
  }
  return ret;
}

// ---- vcgen_stroke / math_stroke (agg_vcgen_stroke.cpp, agg_math_stroke.h) ---------------------------
DEV double pdist(P a, P b) { return sqrt((b.x - a.x) * (b.x - a.x) + (b.y - a.y) * (b.y - a.y)); }

DEV double cross_product(double x1, double y1, double x2, double y2, double x, double y) {
  return (x - x2) * (y2 - y1) - (y - y2) * (x2 - x1);
}

struct Out {
  P v[kMaxV];
  int n = 0;
  bool overflow = false;
  DEV void add(double x, double y) {
    if (n < kMaxV) v[n++] = P{x, y};
    else overflow = true;
  }
};

DEV void calc_miter(Out& o, P v0, P v1, P v2, double dx1, double dy1, double dx2, double dy2, bool revert,
                    double mlimit, double hw) {
  const double lim = hw * mlimit;
  bool exceeded = true;
  // calc_intersection
  const double ax = v0.x + dx1, ay = v0.y - dy1, bx = v1.x + dx1, by = v1.y - dy1;
  const double cx = v1.x + dx2, cy = v1.y - dy2, ddx = v2.x + dx2, ddy = v2.y - dy2;
  const double num = (ay - cy) * (ddx - cx) - (ax - cx) * (ddy - cy);
  const double den = (bx - ax) * (ddy - cy) - (by - ay) * (ddx - cx);
  const bool ok = fabs(den) >= 1.0e-30;
  if (ok) {
    const double rr = num / den;
    const double xi = ax + rr * (bx - ax), yi = ay + rr * (by - ay);
    if (pdist(v1, P{xi, yi}) <= lim) {
      o.add(xi, yi);
      exceeded = false;
    }
  } else {
    const double x2 = v1.x + dx1, y2 = v1.y - dy1;
    if ((cross_product(v0.x, v0.y, v1.x, v1.y, x2, y2) < 0.0) ==
        (cross_product(v1.x, v1.y, v2.x, v2.y, x2, y2) < 0.0)) {
      o.add(v1.x + dx1, v1.y - dy1);
      exceeded = false;
    }
  }
  if (exceeded) {
    // miter_join_revert (inner joins): bevel. The outer miter of an axis-aligned rectangle stays
    // inside its limit (sqrt 2 < width in px); a failed outer intersection is treated the same.
    o.add(v1.x + dx1, v1.y - dy1);
    o.add(v1.x + dx2, v1.y - dy2);
  }
  (void)revert;
}

DEV void calc_join(Out& o, P v0, P v1, P v2, double len1, double len2, double hw, double miter_limit) {
  const double dx1 = hw * (v1.y - v0.y) / len1;
  const double dy1 = hw * (v1.x - v0.x) / len1;
  const double dx2 = hw * (v2.y - v1.y) / len2;
  const double dy2 = hw * (v2.x - v1.x) / len2;
  const double cp = cross_product(v0.x, v0.y, v1.x, v1.y, v2.x, v2.y);
  if (cp > 1e-14) {  // inner join (width > 0): inner_miter, limit max(min(len) / w, 1.01)
    double limit = ((len1 < len2) ? len1 : len2) / hw;
    if (limit < 1.01) limit = 1.01;
    calc_miter(o, v0, v1, v2, dx1, dy1, dx2, dy2, true, limit, hw);
  } else {
    calc_miter(o, v0, v1, v2, dx1, dy1, dx2, dy2, false, miter_limit, hw);
  }
}

DEV void calc_cap(Out& o, P v0, P v1, double len, double hw) {  // butt cap
  double dx1 = (v1.y - v0.y) / len;
  double dy1 = (v1.x - v0.x) / len;
  dx1 *= hw;
  dy1 *= hw;
  o.add(v0.x - dx1, v0.y + dy1);
  o.add(v0.x + dx1, v0.y - dy1);
}

// vertex_sequence<vertex_dist>::add + close(closed)
DEV int dedup(P* s, int n_in, bool closed) {
  int n = 0;
  for (int i = 0; i < n_in; ++i) {
    if (n > 1 && !(pdist(s[n - 2], s[n - 1]) > 1e-14)) --n;
    s[n++] = s[i];
  }
  while (n > 1 && !(pdist(s[n - 2], s[n - 1]) > 1e-14)) {
    s[n - 2] = s[n - 1];
    --n;
  }
  if (closed)
    while (n > 1 && !(pdist(s[n - 1], s[0]) > 1e-14)) --n;
  return n;
}

__global__ __launch_bounds__(64) void box_outline_k(const float* __restrict__ boxes, const int32_t* __restrict__ nbox,
                                                   int max_boxes, int B, int H, int W, double td_sx, double td_tx,
                                                   double td_sy, double td_ty, double width_px,
                                                   BoxOutline* __restrict__ out, int32_t* __restrict__ err) {
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (int64_t)B * max_boxes) return;
  const int b = (int)(id / max_boxes), i = (int)(id % max_boxes);
  if (i >= nbox[b]) return;
  BoxOutline& ol = out[id];
  const float* bx = boxes + id * 4;
  // Rectangle((x0, y0), x1 - x0, y1 - y0) on the float32 box: far corner = x0 + width in f32
  const float x0f = bx[0], y0f = bx[1];
  const float wf = bx[2] - bx[0], hf = bx[3] - bx[1];
  const float x1f = x0f + wf, y1f = y0f + hf;
  // BboxTransformTo(bbox) composed with transData (np.dot), then Agg's flip
  const double bw = (double)x1f - (double)x0f, bh = (double)y1f - (double)y0f;
  const double sx = td_sx * bw, tx = td_sx * (double)x0f + td_tx;
  double sy = td_sy * bh, ty = td_sy * (double)y0f + td_ty;
  ty = -ty + (double)H;
  sy = -sy;
  const double X0 = tx, X1 = sx + tx, Y0 = ty, Y1 = sy + ty;
  const P rect[4] = {{X0, Y0}, {X1, Y0}, {X1, Y1}, {X0, Y1}};
  // PathClipper
  const double r[4] = {-1.0, -1.0, W + 1.0, H + 1.0};
  P sub[kMaxSub][5];
  int sub_n[kMaxSub], n_sub = 0;
  bool sub_closed[kMaxSub] = {false, false, false, false};
  bool moveto = true, was_clipped = false;
  for (int k = 0; k < 4; ++k) {
    double ax = rect[k].x, ay = rect[k].y, cx = rect[(k + 1) & 3].x, cy = rect[(k + 1) & 3].y;
    const int moved = clip_line_segment(&ax, &ay, &cx, &cy, r);
    was_clipped = was_clipped || moved != 0;
    if (moved < 4) {
      if ((moved & 1) || moveto) {
        sub[n_sub][0] = P{ax, ay};
        sub_n[n_sub] = 1;
        ++n_sub;
      }
      sub[n_sub - 1][sub_n[n_sub - 1]++] = P{cx, cy};
      if (k == 3 && !was_clipped) sub_closed[n_sub - 1] = true;
      moveto = false;
    }
  }
  // PathSnapper, then stroke each subpath
  const double snapv = (agg_iround(width_px) % 2) ? 0.5 : 0.0;
  const double hw = width_px * 0.5;
  Out o;
  int cstart[kMaxC + 1], nc = 0;
  for (int s = 0; s < n_sub; ++s) {
    P* v = sub[s];
    for (int j = 0; j < sub_n[s]; ++j) {
      v[j].x = floor(v[j].x + 0.5) + snapv;
      v[j].y = floor(v[j].y + 0.5) + snapv;
    }
    bool closed = sub_closed[s];
    const int n = dedup(v, sub_n[s], closed);
    if (closed && n < 3) closed = false;
    if (n < 2) continue;
    if (closed) {
      double dist[5];
      for (int j = 0; j < n; ++j) dist[j] = pdist(v[j], v[(j + 1) % n]);
      cstart[nc++] = o.n;
      for (int j = 0; j < n; ++j)
        calc_join(o, v[(j + n - 1) % n], v[j], v[(j + 1) % n], dist[(j + n - 1) % n], dist[j], hw, width_px);
      cstart[nc++] = o.n;
      for (int j = n - 1; j >= 0; --j)
        calc_join(o, v[(j + 1) % n], v[j], v[(j + n - 1) % n], dist[j], dist[(j + n - 1) % n], hw, width_px);
    } else {
      double dist[5];
      for (int j = 0; j + 1 < n; ++j) dist[j] = pdist(v[j], v[j + 1]);
      cstart[nc++] = o.n;
      calc_cap(o, v[0], v[1], dist[0], hw);
      for (int j = 1; j + 1 < n; ++j) calc_join(o, v[j - 1], v[j], v[j + 1], dist[j - 1], dist[j], hw, width_px);
      calc_cap(o, v[n - 1], v[n - 2], dist[n - 2], hw);
      for (int j = n - 2; j > 0; --j) calc_join(o, v[j + 1], v[j], v[j - 1], dist[j], dist[j - 1], hw, width_px);
    }
  }
  cstart[nc] = o.n;
  if (o.overflow || nc > kMaxC) {
    atomicOr(err, 1);
    nc = 0;
  }
  ol.n_contours = nc;
  ol.n_vert = nc ? o.n : 0;
  int ex0 = INT32_MAX, ex1 = INT32_MIN, ey0 = INT32_MAX, ey1 = INT32_MIN;
  for (int j = 0; j < ol.n_vert; ++j) {
    const int xi = agg_iround(o.v[j].x * 256.0), yi = agg_iround(o.v[j].y * 256.0);
    ol.x[j] = xi;
    ol.y[j] = yi;
    ex0 = min(ex0, xi >> 8);
    ex1 = max(ex1, xi >> 8);
    ey0 = min(ey0, yi >> 8);
    ey1 = max(ey1, yi >> 8);
  }
  for (int k = 0; k <= nc; ++k) ol.start[k] = cstart[k];
  ol.ex0 = ex0;
  ol.ex1 = ex1;
  ol.ey0 = ol.n_vert ? ey0 : 1;
  ol.ey1 = ol.n_vert ? ey1 : 0;
}

// ---- rasterizer_cells_aa (agg_rasterizer_cells_aa.h), one row -----------------------------------------
struct CellSink {
  int32_t* ex;
  int32_t* cover;
  int32_t* area;
  int32_t* count;
  int32_t* err;
  DEV void emit(int x, int c, int a) {
    if (c == 0 && a == 0) return;
    const int slot = atomicAdd(count, 1);
    if (slot < kMaxCells) {
      ex[slot] = x;
      cover[slot] = c;
      area[slot] = a;
    } else {
      atomicOr(err, 2);
    }
  }
};

DEV void floor_divmod(int64_t p, int64_t d, int64_t* q, int64_t* m) {
  int64_t qq = p / d, mm = p % d;
  if (mm < 0) {
    --qq;
    mm += d;
  }
  *q = qq;
  *m = mm;
}

DEV void render_hline(int ey, int x1, int y1, int x2, int y2, CellSink& sink) {
  const int ex1 = x1 >> 8, ex2 = x2 >> 8;
  const int fx1 = x1 & 255, fx2 = x2 & 255;
  (void)ey;
  if (y1 == y2) return;
  if (ex1 == ex2) {
    const int delta = y2 - y1;
    sink.emit(ex1, delta, (fx1 + fx2) * delta);
    return;
  }
  int64_t p = (int64_t)(256 - fx1) * (y2 - y1);
  int first = 256, incr = 1;
  int64_t dx = (int64_t)x2 - x1;
  if (dx < 0) {
    p = (int64_t)fx1 * (y2 - y1);
    first = 0;
    incr = -1;
    dx = -dx;
  }
  int64_t delta, mod;
  floor_divmod(p, dx, &delta, &mod);
  sink.emit(ex1, (int)delta, (fx1 + first) * (int)delta);
  int ex = ex1 + incr;
  int64_t yy = y1 + delta;
  if (ex != ex2) {
    int64_t lift, rem;
    floor_divmod((int64_t)256 * (y2 - yy + delta), dx, &lift, &rem);
    mod -= dx;
    while (ex != ex2) {
      int64_t d = lift;
      mod += rem;
      if (mod >= 0) {
        mod -= dx;
        ++d;
      }
      sink.emit(ex, (int)d, 256 * (int)d);
      yy += d;
      ex += incr;
    }
  }
  const int dl = (int)(y2 - yy);
  sink.emit(ex2, dl, (fx2 + 256 - first) * dl);
}

// the cells rasterizer_cells_aa::line(x1, y1, x2, y2) adds in cell row `row`
DEV void line_row(int x1, int y1, int x2, int y2, int row, CellSink& sink) {
  int ey1 = y1 >> 8;
  const int ey2 = y2 >> 8;
  const int fy1 = y1 & 255, fy2 = y2 & 255;
  if (row < min(ey1, ey2) || row > max(ey1, ey2)) return;
  if (ey1 == ey2) {
    render_hline(ey1, x1, fy1, x2, fy2, sink);
    return;
  }
  const int64_t dx = (int64_t)x2 - x1;
  int64_t dy = (int64_t)y2 - y1;
  int incr = 1;
  if (dx == 0) {
    const int ex = x1 >> 8;
    const int two_fx = (x1 - (ex << 8)) << 1;
    int first = 256;
    if (dy < 0) {
      first = 0;
      incr = -1;
    }
    int delta;
    if (row == ey1) delta = first - fy1;
    else if (row == ey2) delta = fy2 - 256 + first;
    else delta = first + first - 256;
    sink.emit(ex, delta, two_fx * delta);
    return;
  }
  int64_t p = (int64_t)(256 - fy1) * dx;
  int first = 256;
  if (dy < 0) {
    p = (int64_t)fy1 * dx;
    first = 0;
    incr = -1;
    dy = -dy;
  }
  int64_t delta, mod;
  floor_divmod(p, dy, &delta, &mod);
  int x_from = (int)(x1 + delta);
  if (row == ey1) {
    render_hline(ey1, x1, fy1, x_from, first, sink);
    return;
  }
  ey1 += incr;
  if (ey1 != ey2) {
    int64_t lift, rem;
    floor_divmod((int64_t)256 * dx, dy, &lift, &rem);
    mod -= dy;
    while (ey1 != ey2) {
      int64_t d = lift;
      mod += rem;
      if (mod >= 0) {
        mod -= dy;
        ++d;
      }
      const int x_to = (int)(x_from + d);
      if (ey1 == row) {
        render_hline(ey1, x_from, 256 - first, x_to, first, sink);
        return;
      }
      x_from = x_to;
      ey1 += incr;
    }
  }
  render_hline(ey1, x_from, 256 - first, x2, fy2, sink);
}

DEV int mult_cover(int a, int b) {
  const int t = a * b + 128;
  return ((t >> 8) + t) >> 8;
}

// one wave per (image, canvas row)
__global__ __launch_bounds__(64) void box_rows_k(const uint8_t* __restrict__ src, int64_t sb, int64_t sc,
                                                 int64_t sy, int64_t sx, int H, int W,
                                                 const int32_t* __restrict__ rows, const int32_t* __restrict__ cols,
                                                 const BoxOutline* __restrict__ outlines,
                                                 const int32_t* __restrict__ nbox, const uint8_t* __restrict__ colors,
                                                 int max_boxes, int a8, uint8_t* __restrict__ out,
                                                 int32_t* __restrict__ err) {
  __shared__ uint8_t row[3][kMaxW];
  __shared__ int32_t c_ex[kMaxCells], c_cov[kMaxCells], c_area[kMaxCells];
  __shared__ int32_t n_cells;
  const int r = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
  const uint8_t* s = src + b * sb + (int64_t)rows[r] * sy;
  for (int x = lane; x < W; x += 64) {
    const int64_t o = (int64_t)cols[x] * sx;
    row[0][x] = s[o];
    row[1][x] = s[sc + o];
    row[2][x] = s[2 * sc + o];
  }
  const int nb = nbox[b];
  for (int i = 0; i < nb; ++i) {
    const BoxOutline& ol = outlines[(int64_t)b * max_boxes + i];
    if (r < ol.ey0 || r > ol.ey1) continue;  // uniform across the wave
    if (lane == 0) n_cells = 0;
    __syncthreads();
    CellSink sink{c_ex, c_cov, c_area, &n_cells, err};
    for (int e = lane; e < ol.n_vert; e += 64) {
      int k = 0;
      while (e >= ol.start[k + 1]) ++k;
      const int e2 = (e + 1 < ol.start[k + 1]) ? e + 1 : ol.start[k];
      line_row(ol.x[e], ol.y[e], ol.x[e2], ol.y[e2], r, sink);
    }
    __syncthreads();
    const int nc = min(n_cells, kMaxCells);
    const int x_lo = max(ol.ex0, 0), x_hi = min(ol.ex1, W - 1);
    const uint8_t* col = colors + ((int64_t)b * max_boxes + i) * 3;
    for (int x = x_lo + lane; x <= x_hi; x += 64) {
      int cov = 0, area = 0;
      for (int j = 0; j < nc; ++j) {
        const int cx = c_ex[j];
        if (cx <= x) cov += c_cov[j];
        if (cx == x) area += c_area[j];
      }
      int a = ((cov << 9) - area) >> 9;
      if (a < 0) a = -a;
      if (a > 255) a = 255;
      const int al = mult_cover(a8, a);
      if (al == 0) continue;
      for (int c = 0; c < 3; ++c) {
        const int cr = col[c];
        if (a8 == 255 && a == 255) {
          row[c][x] = (uint8_t)cr;
        } else {
          const int pr = (int)row[c][x] * 255;
          const int A = ((al + 255) << 8) - al * 255;
          row[c][x] = (uint8_t)((((cr << 8) - pr) * al + (pr << 8)) / A);
        }
      }
    }
    __syncthreads();
  }
  __syncthreads();
  uint8_t* d = out + ((int64_t)b * 3 * H + r) * W;
  for (int x = lane; x < W; x += 64) {
    d[x] = row[0][x];
    d[(int64_t)H * W + x] = row[1][x];
    d[(int64_t)2 * H * W + x] = row[2][x];
  }
}

// ---- host geometry: matplotlib's transforms for a VisImage of H x W (oracle axes_transform etc.) -------
struct Aff {
  double sx, tx, sy, ty;
};
Aff dot(Aff b, Aff a) { return Aff{b.sx * a.sx, b.sx * a.tx + b.tx, b.sy * a.sy, b.sy * a.ty + b.ty}; }

void axes_transform(int H, int W, Aff* td, double* axb) {
  const double dpi = 100.0;
  const double w_in = (W + 1e-2) / dpi, h_in = (H + 1e-2) / dpi;
  const double fw = w_in * dpi, fh = h_in * dpi;
  const double fig_aspect = fh / fw;
  const double box_aspect = 1.0 * (std::fabs(0.0 - H) / std::fabs(W - 0.0));
  double hh = 1.0 * box_aspect / fig_aspect, ww;
  if (hh <= 1.0) {
    ww = 1.0;
  } else {
    ww = 1.0 * fig_aspect / box_aspect;
    hh = 1.0;
  }
  const double ox = (0.0 + 0.5 * (1.0 - ww)) - 0.0;
  const double oy = (0.0 + 0.5 * (1.0 - hh)) - 0.0;
  const Aff sub{fw - 0.0, 0.0, fh - 0.0, 0.0};
  const double ax0 = sub.sx * (0.0 + ox) + sub.tx, ay0 = sub.sy * (0.0 + oy) + sub.ty;
  const double ax1 = sub.sx * (ww + ox) + sub.tx, ay1 = sub.sy * (hh + oy) + sub.ty;
  const double inw = W - 0.0, inh = 0.0 - H;
  const double xs = 1.0 / inw, ys = 1.0 / inh;
  const Aff frm{xs, -0.0 * xs, ys, -(double)H * ys};
  const Aff to{ax1 - ax0, ax0, ay1 - ay0, ay0};
  *td = dot(to, frm);
  axb[0] = ax0;
  axb[1] = ay0;
  axb[2] = ax1;
  axb[3] = ay1;
}

std::vector<int> dda2(int y1, int y2, int count) {
  const int cnt = count > 0 ? count : 1;
  int lft = (y2 - y1) / cnt, rem = (y2 - y1) % cnt;
  int mod = rem, y = y1;
  if (mod <= 0) {
    mod += count;
    rem += count;
    --lft;
  }
  mod -= count;
  std::vector<int> out((size_t)count);
  for (int i = 0; i < count; ++i) {
    out[(size_t)i] = y;
    mod += rem;
    y += lft;
    if (mod > 0) {
      mod -= cnt;
      ++y;
    }
  }
  return out;
}

}  // namespace

extern "C" int cullavo_visimage_geometry(int H, int W, int32_t* rows, int32_t* cols, double* trans4) {
  CV_REQUIRE(H > 0 && W > 0 && rows != nullptr && cols != nullptr && trans4 != nullptr, CULLAVO_EINVAL,
             "visimage geometry needs H, W > 0 and output buffers");
  Aff td;
  double axb[4];
  axes_transform(H, W, &td, axb);
  trans4[0] = td.sx;
  trans4[1] = td.tx;
  trans4[2] = td.sy;
  trans4[3] = td.ty;
  // imshow's resample affine (image.py _make_image, origin "upper", extent (0, W, H, 0))
  const Aff a1{1.0, 0.0, -1.0, (0.0 - H) * -1.0};
  const Aff a2{(double)W / W, 0.0 * ((double)W / W) + 0.0, (0.0 - H) / H, 0.0 + (double)H};
  Aff t = dot(dot(td, a2), a1);
  const double p0x = td.sx * 0.0 + td.tx, p0y = td.sy * (double)H + td.ty;
  const double p1x = td.sx * (double)W + td.tx, p1y = td.sy * 0.0 + td.ty;
  const double cx0 = std::max(std::min(p0x, p1x), std::min(axb[0], axb[2]));
  const double cx1 = std::min(std::max(p0x, p1x), std::max(axb[0], axb[2]));
  const double cy0 = std::max(std::min(p0y, p1y), std::min(axb[1], axb[3]));
  const double cy1 = std::min(std::max(p0y, p1y), std::max(axb[1], axb[3]));
  t = dot(Aff{1.0, -cx0 * 1.0, 1.0, -cy0 * 1.0}, t);
  const double owb = (cx1 - cx0) * 1.0, ohb = (cy1 - cy0) * 1.0;
  int ow, oh;
  if (std::fmod(owb, 1.0) != 0.0 || std::fmod(ohb, 1.0) != 0.0) {
    ow = (int)std::ceil(owb);
    oh = (int)std::ceil(ohb);
    t = dot(Aff{1.0 + (ow - owb) / owb, 0.0, 1.0 + (oh - ohb) / ohb, 0.0}, t);
  } else {
    ow = (int)owb;
    oh = (int)ohb;
  }
  CV_REQUIRE(ow >= W && oh >= H + 1, CULLAVO_EUNSUPPORTED, "unexpected VisImage resample buffer size");
  // agg::trans_affine::invert, span_interpolator_linear + dda2, span_image_filter_rgba_nn
  const double d = 1.0 / (t.sx * t.sy - 0.0 * 0.0);
  const double ishx = -0.0 * d, ishy = -0.0 * d;
  const double isx = t.sy * d, isy = t.sx * d;
  const double itx = -t.tx * isx - t.ty * ishx;
  const double ity = -t.tx * ishy - t.ty * isy;
  const double xa = 0.5 * isx + 0.5 * ishx + itx;
  const double xb = (0.5 + ow) * isx + 0.5 * ishx + itx;
  const std::vector<int> xs = dda2(agg_iround(xa * 256.0), agg_iround(xb * 256.0), ow);
  for (int x = 0; x < W; ++x) {
    cols[x] = xs[(size_t)x] >> 8;
    CV_REQUIRE(cols[x] >= 0 && cols[x] < W, CULLAVO_EUNSUPPORTED, "VisImage column map out of range");
  }
  for (int r = 0; r < H; ++r) {
    const double yy = 0.5 * ishy + ((double)(oh - 2 - r) + 0.5) * isy + ity;
    rows[r] = agg_iround(yy * 256.0) >> 8;
    CV_REQUIRE(rows[r] >= 0 && rows[r] < H, CULLAVO_EUNSUPPORTED, "VisImage row map out of range");
  }
  return CULLAVO_OK;
}

extern "C" size_t cullavo_draw_boxes_workspace(int B, int max_boxes) {
  return 256 + sizeof(BoxOutline) * (size_t)std::max(B, 0) * (size_t)std::max(max_boxes, 1);
}

extern "C" int cullavo_draw_boxes(const uint8_t* images, int B, int C, int H, int W, int64_t sb, int64_t sc, int64_t sy,
                                  int64_t sx, const int32_t* rows, const int32_t* cols, const float* boxes,
                                  const int32_t* nbox, const uint8_t* colors, int max_boxes, double td_sx,
                                  double td_tx, double td_sy, double td_ty, double width_px, int alpha8,
                                  void* workspace, uint8_t* out, void* stream) {
  CV_REQUIRE(B >= 0 && C == 3 && H > 0 && W > 0, CULLAVO_EINVAL, "draw_boxes needs RGB images [B, 3, H, W]");
  CV_REQUIRE(W <= kMaxW, CULLAVO_EUNSUPPORTED, "draw_boxes: image wider than 8192 px");
  CV_REQUIRE(max_boxes >= 0 && alpha8 >= 0 && alpha8 <= 255 && width_px > 0.0, CULLAVO_EINVAL,
             "draw_boxes: bad box count, alpha or line width");
  if (B == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  int32_t* err = reinterpret_cast<int32_t*>(workspace);
  BoxOutline* outlines = reinterpret_cast<BoxOutline*>(reinterpret_cast<char*>(workspace) + 256);
  if (hipMemsetAsync(err, 0, sizeof(int32_t), s) != hipSuccess) return cullavo_check_launch("draw_boxes memset");
  if (max_boxes > 0) {
    const int64_t n = (int64_t)B * max_boxes;
    box_outline_k<<<(unsigned)cdiv(n, 64), 64, 0, s>>>(boxes, nbox, max_boxes, B, H, W, td_sx, td_tx, td_sy, td_ty,
                                                     width_px, outlines, err);
  }
  box_rows_k<<<dim3((unsigned)H, (unsigned)B), 64, 0, s>>>(images, sb, sc, sy, sx, H, W, rows, cols, outlines, nbox,
                                                          colors, max_boxes, alpha8, out, err);
  return cullavo_check_launch("draw_boxes");
}
