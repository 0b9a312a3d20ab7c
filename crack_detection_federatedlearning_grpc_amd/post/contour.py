"""Crack post-processing: threshold + contours + area / perimeter / approximations (native, csrc/native/contour.cpp).

Reference ``contour(img)`` (test/Segmentation2.py:114-141) - threshold 127, findContours(RETR_TREE,
CHAIN_APPROX_SIMPLE), contourArea/arcLength of ``contours[0]``, approxPolyDP at 1 % and 10 % of the perimeter,
drawn to contour/img{1,2,3}.jpg. ``client_fit_model.py:215`` calls an undefined ``self.contour``; here
it is a real function returning the numbers instead of printing them.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from .._native_loader import native


def find_contours(gray: np.ndarray, thresh: int = 127, simple: bool = True) -> Tuple[List[np.ndarray], np.ndarray]:
    cs, hier, _ = native().contour.find_contours(np.ascontiguousarray(gray, np.uint8), thresh, simple)
    return cs, hier


def contour_area(pts: np.ndarray) -> float:
    return native().contour.contour_area(np.asarray(pts, np.int32), False)


def arc_length(pts: np.ndarray, closed: bool = True) -> float:
    return native().contour.arc_length(np.asarray(pts, np.int32), closed)


def approx_poly_dp(pts: np.ndarray, epsilon: float, closed: bool = True) -> np.ndarray:
    return native().contour.approx_poly_dp(np.asarray(pts, np.int32), float(epsilon), closed)


def crack_metrics(pred_u8: np.ndarray, thresh: int = 127) -> Dict[str, float]:
    """Metrics for one predicted mask (uint8, 0..255 gray or HxWx3 BGR/RGB)."""
    g = pred_u8
    if g.ndim == 3:   # cv2.COLOR_BGR2GRAY weights
        g = np.clip(0.114 * g[..., 0] + 0.587 * g[..., 1] + 0.299 * g[..., 2] + 0.5, 0, 255).astype(np.uint8)
    cs, hier = find_contours(g, thresh)
    areas = [contour_area(c) for c in cs]
    perims = [arc_length(c, True) for c in cs]
    out = {"count": float(len(cs)), "pixels": float((g > thresh).sum())}
    if cs:
        out.update(first_area=areas[0], first_perimeter=perims[0], total_area=float(sum(areas)),
                   total_perimeter=float(sum(perims)), max_area=float(max(areas)),
                   length_estimate=float(sum(perims)) / 2.0,
                   approx1_points=float(len(approx_poly_dp(cs[0], 0.01 * perims[0]))),
                   approx2_points=float(len(approx_poly_dp(cs[0], 0.1 * perims[0]))))
    return out
