import numpy as np
import pytest

from crack_detection_federatedlearning_grpc_amd._native_loader import native
from crack_detection_federatedlearning_grpc_amd.data.folder import load_folder_dataset
from crack_detection_federatedlearning_grpc_amd.data.synthetic import make_synthetic, reference_split
from crack_detection_federatedlearning_grpc_amd.train.local import epoch_batches


def _np_bilinear(a, h, w):
    sh, sw = a.shape[:2]
    out = np.zeros((h, w) + a.shape[2:], np.float32)
    for y in range(h):
        sy = (y + 0.5) * sh / h - 0.5
        iy = int(np.floor(sy)); b = sy - iy
        if iy < 0: iy, b = 0, 0.0
        if iy >= sh - 1: iy, b = sh - 1, 0.0
        iy1 = min(iy + 1, sh - 1)
        for x in range(w):
            sx = (x + 0.5) * sw / w - 0.5
            ix = int(np.floor(sx)); t = sx - ix
            if ix < 0: ix, t = 0, 0.0
            if ix >= sw - 1: ix, t = sw - 1, 0.0
            ix1 = min(ix + 1, sw - 1)
            top = a[iy, ix] * (1 - t) + a[iy, ix1] * t
            bot = a[iy1, ix] * (1 - t) + a[iy1, ix1] * t
            out[y, x] = top * (1 - b) + bot * b
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def test_native_resize_matches_numpy_reference():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    for h, w in [(16, 16), (64, 80), (37, 53)]:
        got = native().resize_bilinear(a, h, w, 3)
        ref = _np_bilinear(a.astype(np.float32), h, w)
        assert np.abs(got.astype(int) - ref.astype(int)).max() <= 1
    assert np.array_equal(native().resize_bilinear(a, 37, 53, 1), a)


def test_reference_split_semantics():
    import random
    idx = list(range(10))
    random.Random(1337).shuffle(idx)
    tr, va = reference_split(10, 6)
    assert list(tr) == idx[:6] and list(va) == idx[6:]       # client: FIRST n are train
    tr2, va2 = reference_split(10, 4, client_first=False)
    assert list(va2) == idx[-4:]                              # test/Segmentation.py: LAST n are val


def test_epoch_batches_sequence_semantics():
    idx = np.arange(50)
    b = epoch_batches(idx, 16, 0, seed=1)
    assert b.shape == (3, 16)                                 # len = n // batch, remainder dropped
    assert sorted(b.reshape(-1).tolist()) == list(range(48))
    assert epoch_batches(idx, 16, 7, seed=1).shape == (7, 16)


def test_synthetic_has_cracks_and_texture():
    d = make_synthetic(6, 64, seed=5, split=4)
    assert d.images.shape == (6, 64, 64, 3) and d.masks.shape == (6, 64, 64)
    assert 0.002 < d.masks.mean() < 0.3
    crack = d.images[..., 1][d.masks > 0].mean()
    bg = d.images[..., 1][d.masks == 0].mean()
    assert crack < bg - 20
    assert len(d.train_idx) == 4 and len(d.val_idx) == 2


def test_folder_dataset(tmp_path):
    from PIL import Image
    (tmp_path / "img").mkdir()
    (tmp_path / "mask").mkdir()
    d = make_synthetic(5, 48, seed=2)
    for i in range(5):
        Image.fromarray(d.images[i]).save(tmp_path / "img" / f"c{i:03d}.jpg", quality=95)
        Image.fromarray(d.masks[i] * 255).save(tmp_path / "mask" / f"c{i:03d}.jpg", quality=95)
    (tmp_path / "mask" / ".hidden.jpg").write_bytes(b"x")
    ds = load_folder_dataset(str(tmp_path / "img"), str(tmp_path / "mask"), 32, split=3)
    assert ds.images.shape == (5, 32, 32, 3) and ds.masks.shape == (5, 32, 32)
    assert set(np.unique(ds.masks)) <= {0, 1}
    assert len(ds.train_idx) == 3 and len(ds.val_idx) == 2
