#!/usr/bin/env python3
"""MNIST IDX -> PNG tree (the dataset layout DLI ingests), like the reference
``convert_mnist.py`` but with the CLI its commented-out usage describes (Q12):

    python convert_mnist.py <input_path> <output_path> [--tfrecord] [--channels 3]

For ``training`` and ``testing`` it reads ``{train,t10k}-{images-idx3,labels-idx1}-ubyte``
(optionally .gz) and writes ``<output_path>/<dataset>/{0..9}/<index>.png``
(``convert_mnist.py:59-70``).  ``--tfrecord`` additionally writes the TFRecords
DLI would build from that tree (``image_raw`` + ``label``; ``--channels 3`` gives
the 2352-byte RGB records the reference trainer expects, ``mnist_input.py:13-15``).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402

from distributed_tensorflow_ibm_mnist_amd.data.idx import read, write_dataset  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("input_path")
    ap.add_argument("output_path")
    ap.add_argument("--datasets", default="training,testing")
    ap.add_argument("--tfrecord", action="store_true", help="also write <dataset>.tfrecords")
    ap.add_argument("--channels", type=int, default=3, choices=[1, 3])
    ap.add_argument("--no_png", action="store_true")
    ap.add_argument("--verbose", action="store_true", help="print every file written (reference behaviour)")
    a = ap.parse_args(argv)
    for dataset in a.datasets.split(","):
        labels, data, size, rows, cols = read(dataset, a.input_path)
        out = os.path.join(a.output_path, dataset)
        if not a.no_png:
            write_dataset(labels, data, size, rows, cols, out, verbose=a.verbose)
        if a.tfrecord:
            from distributed_tensorflow_ibm_mnist_amd.data.tfrecord import write_mnist_tfrecords
            imgs = np.asarray(data, dtype=np.uint8).reshape(size, rows * cols, 1)
            if a.channels == 3:
                imgs = np.repeat(imgs, 3, axis=2)
            os.makedirs(a.output_path, exist_ok=True)
            write_mnist_tfrecords(os.path.join(a.output_path, f"{dataset}.tfrecords"), imgs.reshape(size, -1),
                                  labels)
        print(f"{dataset}: {size} images ({rows}x{cols}) -> {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
