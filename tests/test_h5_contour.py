import os
import shutil
import subprocess

import numpy as np
import pytest

from crack_detection_federatedlearning_grpc_amd.ckpt.h5 import (load_optimizer_h5, load_weights_h5, read_h5,
                                                                save_keras_h5, save_weights_h5)
from crack_detection_federatedlearning_grpc_amd.post import contour as C

H5DUMP = "/opt/conda/bin/h5dump"


def test_h5_roundtrip_full_model(tmp_path, table):
    f = table.init_flat(7)
    p = str(tmp_path / "crack_segmentation.h5")
    save_keras_h5(p, table, f, img_size=128, optimizer=(42, f * 0.5, f * f))
    assert np.array_equal(load_weights_h5(p, table), f)
    it, m, v = load_optimizer_h5(p, table)
    assert it == 42 and np.allclose(m[table.trainable_mask() > 0], (f * 0.5)[table.trainable_mask() > 0])
    tree = read_h5(p)
    assert set(tree["attrs"]) >= {"backend", "keras_version", "model_config", "training_config"}
    mw = tree["groups"]["model_weights"]
    assert len(mw["attrs"]["layer_names"]) == len(table.layers)
    assert [w.decode() for w in mw["groups"]["separable_conv2d"]["attrs"]["weight_names"]] == [
        "separable_conv2d/depthwise_kernel:0", "separable_conv2d/pointwise_kernel:0", "separable_conv2d/bias:0"]


def test_h5_weights_only(tmp_path, table):
    f = table.init_flat(8)
    p = str(tmp_path / "w.h5")
    save_weights_h5(p, table, f)
    assert np.array_equal(load_weights_h5(p, table), f)


@pytest.mark.skipif(not os.path.exists(H5DUMP), reason="libhdf5 h5dump not present")
def test_h5_readable_by_libhdf5(tmp_path, table):
    f = table.init_flat(9)
    p = str(tmp_path / "k.h5")
    save_keras_h5(p, table, f)
    r = subprocess.run([H5DUMP, "-H", p], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([H5DUMP, "-d", "/model_weights/conv2d_8/conv2d_8/bias:0", p], capture_output=True, text=True)
    assert r.returncode == 0 and "(0): 0" in r.stdout
    e = table.entry("conv2d_8", "kernel")
    r = subprocess.run([H5DUMP, "-d", "/model_weights/conv2d_8/conv2d_8/kernel:0", "-m", "%.9g", p],
                       capture_output=True, text=True)
    vals = [float(x.split(":")[1].strip().rstrip(",")) for x in r.stdout.splitlines() if "(0,0," in x]
    assert np.allclose(vals, f[e.offset:e.offset + e.size])


def test_contour_square_and_hole():
    img = np.zeros((20, 20), np.uint8)
    img[2:12, 3:13] = 255            # 10x10 filled square
    img[5:8, 6:9] = 0                # 3x3 hole
    cs, hier = C.find_contours(img)
    assert len(cs) == 2
    outer = cs[0]
    assert C.contour_area(outer) == 81.0            # polygon through pixel centres: 9 x 9
    assert C.arc_length(outer) == 36.0
    assert len(outer) == 4                          # CHAIN_APPROX_SIMPLE keeps the corners
    assert hier[1][3] == 0 and hier[0][2] == 1      # hole is a child of the outer border (RETR_TREE)
    m = C.crack_metrics(img)
    assert m["count"] == 2 and m["pixels"] == 91


def test_contour_line_crack():
    img = np.zeros((32, 32), np.uint8)
    for i in range(4, 28):
        img[i, i] = 255
    cs, _ = C.find_contours(img)
    assert len(cs) == 1
    assert C.contour_area(cs[0]) == 0.0
    assert abs(C.arc_length(cs[0]) - 2 * 23 * np.sqrt(2)) < 1e-6
    assert len(C.approx_poly_dp(cs[0], 1.0)) == 2
