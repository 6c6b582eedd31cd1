"""Step-2-pre debugging visualisation (reference cullavo/arch_cullavo.py:376-386): the image of a
record with the generated boxes and their class names drawn the way detectron2's
``Visualizer.overlay_instances(boxes=..., labels=..., assigned_colors=...)`` draws them with
``_default_font_size = 16``, rendered by matplotlib's Agg backend (the renderer detectron2 drives)
and returned as an RGB uint8 array for a PNG.

This is a host-side debugging artefact, like the reference's (which writes it to a fixed path on
its authors' machine); it is not on any training step. The box rasters alone are what
``csrc/boxdraw.hip`` reproduces bit-exactly on the GPU for the step-1 / step-2 prompts; the class
labels need a font rasteriser, so they stay with matplotlib here. detectron2 is absent, so the
parity of this image is unpinned; its geometry follows detectron2's published rules:
largest boxes drawn first, box edges alpha 0.5 and width max(font / 4, 1), a label at the box's
top-left corner, moved below the box (or to its top-right corner at the image bottom) for
objects under 1000 px or 40 px high, font size clip((h / sqrt(HW) - 0.02) / 0.08 + 1, 1.2, 2) x
0.5 x 16, text colour the box colour lightened 70 % and kept >= 0.2 per channel with its largest
channel >= 0.8, on a black box of alpha 0.8.
"""
from __future__ import annotations

import colorsys

import numpy as np

SMALL_OBJECT_AREA = 1000  # detectron2 _SMALL_OBJECT_AREA_THRESH


def _label_color(color):
    import matplotlib.colors as mplc
    h, lum, s = colorsys.rgb_to_hls(*mplc.to_rgb(color))
    rgb = np.array(colorsys.hls_to_rgb(h, min(1.0, max(0.0, lum * 1.7)), s))
    rgb = np.maximum(rgb, 0.2)
    rgb[np.argmax(rgb)] = max(0.8, float(np.max(rgb)))
    return rgb


def render_boxes_and_labels(image, boxes, labels, colors, font_size: float = 16.0) -> np.ndarray:
    """image: [3, H, W] or [H, W, 3] uint8 (tensor or array); boxes [n, 4] x0 y0 x1 y1 in pixels;
    labels: n strings (None: boxes only); colors: n matplotlib colours. Returns [H, W, 3] uint8.
    Raises AssertionError when len(labels) != n, as overlay_instances does."""
    import matplotlib.figure as mplfigure
    from matplotlib.backends.backend_agg import FigureCanvasAgg
    from matplotlib.patches import Rectangle

    img = np.asarray(image.cpu() if hasattr(image, "cpu") else image)
    if img.ndim == 3 and img.shape[0] == 3 and img.shape[-1] != 3:
        img = img.transpose(1, 2, 0)
    img = img.clip(0, 255).astype(np.uint8)
    H, W = img.shape[:2]
    boxes = np.asarray(boxes.cpu() if hasattr(boxes, "cpu") else boxes, dtype=np.float64).reshape(-1, 4)
    n = len(boxes)
    if labels is not None:
        assert len(labels) == n, f"{len(labels)} labels for {n} boxes"
    fig = mplfigure.Figure(frameon=False)
    dpi = fig.get_dpi()
    fig.set_size_inches((W + 1e-2) / dpi, (H + 1e-2) / dpi)
    canvas = FigureCanvasAgg(fig)
    ax = fig.add_axes([0.0, 0.0, 1.0, 1.0])
    ax.axis("off")
    ax.imshow(img, extent=(0, W, H, 0), interpolation="nearest")
    areas = np.prod(boxes[:, 2:] - boxes[:, :2], axis=1)
    for i in np.argsort(-areas, kind="stable").tolist() if n else []:
        x0, y0, x1, y1 = boxes[i]
        ax.add_patch(Rectangle((x0, y0), x1 - x0, y1 - y0, fill=False, edgecolor=colors[i],
                               linewidth=max(font_size / 4, 1), alpha=0.5, linestyle="-"))
        if labels is None:
            continue
        pos, align = (x0, y0), "left"
        if (y1 - y0) * (x1 - x0) < SMALL_OBJECT_AREA or y1 - y0 < 40:
            pos = (x1, y0) if y1 >= H - 5 else (x0, y1)
        ratio = (y1 - y0) / np.sqrt(H * W)
        size = np.clip((ratio - 0.02) / 0.08 + 1, 1.2, 2) * 0.5 * font_size
        ax.text(pos[0], pos[1], labels[i], size=size, family="sans-serif",
                bbox={"facecolor": "black", "alpha": 0.8, "pad": 0.7, "edgecolor": "none"},
                verticalalignment="top", horizontalalignment=align, color=_label_color(colors[i]), zorder=10)
    buf, (w, h) = canvas.print_to_buffer()
    return np.frombuffer(buf, dtype=np.uint8).reshape(h, w, 4)[..., :3].copy()
