"""C17 centralized trainer (test/Segmentation.py) + C18 offline analysis tool (test/Segmentation2.py), CPU path."""
import json
import os

import numpy as np

from crack_detection_federatedlearning_grpc_amd import config
from crack_detection_federatedlearning_grpc_amd.ckpt.h5 import load_optimizer_h5, load_weights_h5, read_h5
from crack_detection_federatedlearning_grpc_amd.post.analyze import analyze, draw_contours, load_weights
from crack_detection_federatedlearning_grpc_amd.train.centralized import CentralizedTrainer, main


def test_centralized_checkpoint_save_and_analyze(tmp_path, table):
    cfg = config.from_args(None, preset="cpu-plumbing", epochs=2, metrics_file=str(tmp_path / "m.jsonl"))
    tr = CentralizedTrainer(cfg)
    ck = str(tmp_path / "crack_segmentation.h5")
    hist = tr.train(2, ck, save_best_only=True)
    assert len(hist) == 2 and all(np.isfinite(h["loss"]) and "val_loss" in h for h in hist)
    assert hist[0].get("checkpoint") == ck                      # first epoch always improves on +inf
    tree = read_h5(ck)
    assert "model_config" in tree["attrs"] and "optimizer_weights" in tree["groups"]
    tr.save(str(tmp_path / "my_model"))
    flat = tr.fit.backend.get_flat()
    assert np.array_equal(load_weights(str(tmp_path / "my_model"), table), flat)
    it, m, v = load_optimizer_h5(str(tmp_path / "my_model" / "model.h5"), table)
    assert it == 2 * tr.fit.steps and np.abs(m).sum() > 0
    assert np.array_equal(load_weights_h5(str(tmp_path / "my_model" / "model.h5"), table), flat)
    lines = [json.loads(x) for x in open(tmp_path / "m.jsonl")]
    assert [r["epoch"] for r in lines] == [1, 2] and lines[0]["mode"] == "centralized"

    out = tmp_path / "analysis"
    recs = analyze(cfg, str(tmp_path / "my_model"), str(out), count=2, trainer=tr.fit)
    assert len(recs) == 2 and all("iou" in r and "count" in r for r in recs)
    for i in (1, 2):
        assert (out / f"pred{i}.png").exists() and (out / "contour" / f"img{i}.png").exists()
    assert json.load(open(out / "analysis.json")) == recs


def test_draw_contours_marks_the_boundary():
    prob = np.zeros((32, 32), np.uint8)
    prob[8:20, 10:14] = 255
    img = np.zeros((32, 32, 3), np.uint8)
    out = draw_contours(img, prob)
    red = (out[..., 0] == 255) & (out[..., 1] == 0)
    assert red[8, 10] and red[19, 13] and not red[14, 11] and not red[0, 0]


def test_centralized_cli(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    assert main(["--preset", "cpu-plumbing", "--epochs", "1", "--checkpoint", "ck.h5", "--save-dir", "mm"]) == 0
    assert os.path.exists("ck.h5") and os.path.exists("mm/model.h5") and os.path.exists("mm/weights.pickle")
