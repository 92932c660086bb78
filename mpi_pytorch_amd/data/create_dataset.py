"""Offline dataset sampling (reference: ``/root/reference/create_dataset.py:17-66``).

``metadata.json`` (COCO-style ``images`` + ``annotations``, ISO-8859-1) -> merge on ``id``
-> ``sample(N_IMAGES, random_state=0)`` -> 80/20 ``train_test_split`` -> ``data/*.csv``
-> copy the image files into ``data/img/{train,test}/``.

Differences: the split takes a seed (the reference's is unseeded), paths are arguments,
copying is parallel and optional (``--no-copy``), and ``--make-metadata N`` writes a small
synthetic ``metadata.json`` (+ JPEGs) so the whole flow can be exercised offline.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

import numpy as np
import pandas as pd


def read_json(input_file: str):
    """Read the annotation JSON (ISO-8859-1, like the reference)."""
    with open(input_file, "r", encoding="ISO-8859-1") as f:
        return json.load(f)


def create_dataframe(ann_file) -> pd.DataFrame:
    img = pd.DataFrame(ann_file["images"])
    ann = pd.DataFrame(ann_file["annotations"])
    if "image_id" in ann.columns:
        ann = ann.drop(columns="image_id")
    return img.merge(ann, on="id")


def copy_file(src_root: str, rel: str, dst_root: str, mode: str) -> None:
    dst = os.path.join(dst_root, "img", mode, rel)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    shutil.copy2(os.path.join(src_root, rel), dst)


def make_synthetic_metadata(root: str, n: int, num_classes: int = 64500, seed: int = 0,
                            write_images: bool = True, size=(96, 72)) -> str:
    rng = np.random.default_rng(seed)
    images, anns = [], []
    for i in range(n):
        rel = "images/{:03d}/{:02d}/{}.jpg".format(i % 300, i % 97, 100000 + i)
        images.append({"file_name": rel, "height": size[0], "width": size[1],
                       "id": 100000 + i, "license": 0})
        anns.append({"id": 100000 + i, "image_id": 100000 + i,
                     "category_id": int(rng.integers(0, num_classes)), "institution_id": 0})
        if write_images:
            from PIL import Image
            p = os.path.join(root, rel)
            os.makedirs(os.path.dirname(p), exist_ok=True)
            arr = rng.integers(0, 256, size=(size[0], size[1], 3), dtype=np.uint8)
            Image.fromarray(arr).save(p, quality=90)
    path = os.path.join(root, "metadata.json")
    os.makedirs(root, exist_ok=True)
    with open(path, "w", encoding="ISO-8859-1") as f:
        json.dump({"images": images, "annotations": anns}, f)
    return path


def build(train_dir: str, train_file: str = "metadata.json", n_images: int = 50000,
          out_dir: str = "./data", copy: bool = True, seed: int = 0, workers: int = 8):
    from sklearn.model_selection import train_test_split
    df = create_dataframe(read_json(os.path.join(train_dir, train_file)))
    sample = df.sample(min(n_images, len(df)), random_state=0).reset_index(drop=True)
    train_sample, test_sample = train_test_split(sample, test_size=0.2, random_state=seed)
    os.makedirs(out_dir, exist_ok=True)
    test_sample.to_csv(os.path.join(out_dir, "test_sample.csv"))
    train_sample.to_csv(os.path.join(out_dir, "train_sample.csv"))
    if copy:
        with ThreadPoolExecutor(max_workers=workers) as pool:
            for mode, part in (("test", test_sample), ("train", train_sample)):
                list(pool.map(lambda r: copy_file(train_dir, r, out_dir, mode),
                              part["file_name"].tolist()))
    return train_sample, test_sample


def main(argv: Optional[List[str]] = None) -> None:
    from ..config import Config
    p = argparse.ArgumentParser()
    p.add_argument("--train-dir", default=None)
    p.add_argument("--train-file", default=None)
    p.add_argument("--n-images", type=int, default=None)
    p.add_argument("--out-dir", default="./data")
    p.add_argument("--no-copy", action="store_true")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--make-metadata", type=int, default=0,
                   help="first write a synthetic metadata.json with N images into --train-dir")
    a = p.parse_args(argv)
    cfg = Config.from_env()
    train_dir = a.train_dir or cfg.TRAIN_DIR
    if a.make_metadata:
        make_synthetic_metadata(train_dir, a.make_metadata)
    tr, te = build(train_dir, a.train_file or cfg.TRAIN_FILE, a.n_images or cfg.N_IMAGES,
                   a.out_dir, not a.no_copy, a.seed)
    print("Created train & test samples: {} / {}".format(len(tr), len(te)))
