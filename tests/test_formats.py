"""T1: native formats — crc32c, TFRecord, tf.Example, IDX/PNG, tensor bundle,
checkpoint state, event files."""
import os
import struct

import numpy as np
import pytest

from distributed_tensorflow_ibm_mnist_amd.ops._ext import host


def test_crc32c_known_values():
    H = host()
    assert H.crc32c(b"123456789") == 0xE3069283          # CRC-32C check value
    assert H.crc32c(b"") == 0
    assert H.crc32c(b"\x00" * 32) == 0x8A9136AA          # RFC 3720 test vector
    assert H.crc32c(bytes(range(32))) == 0x46DD794E
    # masked form used by TFRecord / tensor bundles
    c = H.crc32c(b"abc")
    assert H.masked_crc32c(b"abc") == ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def test_tfrecord_roundtrip_and_corruption(tmp_path):
    from distributed_tensorflow_ibm_mnist_amd.data.tfrecord import TFRecordWriter, read_records
    p = str(tmp_path / "x.tfrecords")
    recs = [b"", b"a", os.urandom(1000), b"z" * 70000]
    with TFRecordWriter(p) as w:
        for r in recs:
            w.write(r)
    assert read_records(p) == recs
    raw = bytearray(open(p, "rb").read())
    # frame layout: u64 len | u32 masked crc(len) | data | u32 masked crc(data)
    assert struct.unpack("<Q", raw[:8])[0] == 0
    raw[28] ^= 0xFF   # payload byte of record #1 (record #0 is a 16-byte empty frame)
    open(p, "wb").write(bytes(raw))
    with pytest.raises(RuntimeError):
        read_records(p)


def test_example_codec_and_native_decode(tmp_path):
    from distributed_tensorflow_ibm_mnist_amd.data.tfrecord import (decode_example, encode_example,
                                                                    load_mnist_tfrecords, write_mnist_tfrecords)
    ex = encode_example({"image_raw": b"\x01\x02\x03", "label": 7, "f": [1.5, 2.0]})
    d = decode_example(ex)
    assert d["image_raw"] == b"\x01\x02\x03" and d["label"] == [7] and d["f"] == [1.5, 2.0]
    imgs = np.random.randint(0, 256, (37, 2352), dtype=np.uint8)
    labs = np.random.randint(0, 10, 37)
    p = str(tmp_path / "m.tfrecords")
    write_mnist_tfrecords(p, imgs, labs)
    x, y, c = load_mnist_tfrecords([p])
    assert c == 3 and np.array_equal(x, imgs) and np.array_equal(y, labs)
    with pytest.raises(ValueError):
        load_mnist_tfrecords([str(tmp_path / "missing-*.tfrecords")])


def test_idx_png_roundtrip(tmp_path):
    from distributed_tensorflow_ibm_mnist_amd.data import idx
    imgs = np.random.randint(0, 256, (12, 28, 28), dtype=np.uint8)
    labs = np.arange(12) % 10
    idx.write_idx(str(tmp_path / "train"), imgs, labs)
    lab, pix, n, r, c = idx.read("training", str(tmp_path))
    assert (n, r, c) == (12, 28, 28) and np.array_equal(pix.reshape(n, r, c), imgs) and np.array_equal(lab, labs)
    idx.write_dataset(lab, pix, n, r, c, str(tmp_path / "png"))
    assert sorted(os.listdir(tmp_path / "png")) == [str(i) for i in range(10)]
    back, bl = idx.load_png_tree(str(tmp_path / "png"))
    order = np.lexsort((np.arange(len(bl)), bl))
    # PIL decodes our PNG encoder's output bit-exactly
    from PIL import Image
    im = np.asarray(Image.open(tmp_path / "png" / "3" / "3.png"))
    assert np.array_equal(im, imgs[3])
    assert back.shape == (12, 784) and sorted(bl.tolist()) == sorted(labs.tolist())


def test_crop_or_pad_tf_semantics():
    from distributed_tensorflow_ibm_mnist_amd.data.idx import crop_or_pad
    a = np.arange(30 * 32).reshape(30, 32, 1)
    c = crop_or_pad(a, 28, 28)
    assert np.array_equal(c[..., 0], a[1:29, 2:30, 0])
    b = np.ones((20, 26, 1))
    p = crop_or_pad(b, 28, 28)
    assert p[4:24, 1:27].all() and p.sum() == 20 * 26


def test_bundle_roundtrip_sharded(tmp_path):
    from distributed_tensorflow_ibm_mnist_amd.ckpt.bundle import read_bundle, read_index, write_bundle
    t = {"conv1/weights": np.random.randn(5, 5, 3, 32).astype(np.float32),
         "conv1/biases": np.zeros(32, np.float32),
         "global_step": np.asarray(1234, dtype=np.int64),
         "local3/weights": np.random.randn(300, 40).astype(np.float32)}
    prefix = str(tmp_path / "model.ckpt-1234")
    write_bundle(prefix, t, num_shards=2, shard_of={"local3/weights": 1})
    assert os.path.exists(prefix + ".data-00000-of-00002") and os.path.exists(prefix + ".data-00001-of-00002")
    n, idx = read_index(prefix)
    assert n == 2 and idx["local3/weights"]["shard"] == 1 and idx["global_step"]["shape"] == ()
    assert idx["conv1/weights"]["dtype"] == 1 and idx["global_step"]["dtype"] == 9
    back = read_bundle(prefix)
    for k in t:
        assert np.array_equal(back[k], t[k]) and back[k].dtype == t[k].dtype
    # corrupt a data byte -> checksum error
    d = bytearray(open(prefix + ".data-00001-of-00002", "rb").read())
    d[10] ^= 1
    open(prefix + ".data-00001-of-00002", "wb").write(bytes(d))
    with pytest.raises(IOError):
        read_bundle(prefix)


def test_sstable_many_entries_multiblock():
    H = host()
    ents = [(f"var/{i:06d}".encode(), os.urandom(900)) for i in range(1000)]   # > one 256 KiB block
    blob = H.sstable_build(ents)
    assert H.sstable_parse(blob) == ents
    with pytest.raises(RuntimeError):
        H.sstable_build([(b"b", b""), (b"a", b"")])


def test_saver_max_to_keep_and_state_file(tmp_path):
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import Saver, get_checkpoint_state, latest_checkpoint
    s = Saver(max_to_keep=3)
    for step in (0, 10, 20, 30, 40):
        s.save(str(tmp_path), step, {"w": np.full(4, step, np.float32), "global_step": np.int64(step)})
    st = get_checkpoint_state(str(tmp_path))
    assert st.model_checkpoint_path.endswith("model.ckpt-40")
    assert [os.path.basename(p) for p in st.all_model_checkpoint_paths] == [
        "model.ckpt-20", "model.ckpt-30", "model.ckpt-40"]
    assert not os.path.exists(tmp_path / "model.ckpt-0.index")
    txt = open(tmp_path / "checkpoint").read()
    assert txt.startswith('model_checkpoint_path: "model.ckpt-40"')
    assert Saver.restore(latest_checkpoint(str(tmp_path)))["w"][0] == 40


def test_event_file_roundtrip(tmp_path):
    from distributed_tensorflow_ibm_mnist_amd.obs.events import EventFileWriter, find_event_files, read_events
    w = EventFileWriter(str(tmp_path))
    w.add_scalars({"train loss": 1.25, "train accuracy": 0.5}, 10)
    w.add_histograms({"conv1/weight": np.random.randn(1000)}, 10)
    w.close()
    evs = list(read_events(find_event_files(str(tmp_path))[0]))
    assert evs[0]["file_version"] == "brain.Event:2"
    assert evs[1]["step"] == 10 and evs[1]["values"]["train loss"] == 1.25
    h = evs[2]["values"]["conv1/weight"]
    assert h["num"] == 1000 and sum(h["bucket"]) == 1000


def test_feistel_epoch_permutation_and_sharding():
    """Stateless loader order: every epoch is a full permutation, epochs differ,
    sharded ranks partition each global batch, and seek(step) resumes the order."""
    import torch
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import (DeviceDataset, DeviceLoader,
                                                                         perm_positions)
    for N in (1, 7, 64, 1000, 60000):
        x = perm_positions(0, 3 * N, N, 11)
        for e in range(3):
            assert torch.equal(torch.sort(x[e * N:(e + 1) * N]).values, torch.arange(N))
    a, b = perm_positions(0, 1000, 1000, 1), perm_positions(1000, 1000, 1000, 1)
    assert not torch.equal(a, b) and not torch.equal(a, perm_positions(0, 1000, 1000, 2))
    assert torch.equal(perm_positions(123, 50, 1000, 5), perm_positions(0, 173, 1000, 5)[123:])
    imgs = torch.arange(100, dtype=torch.int64).repeat_interleave(784).view(100, 784).to(torch.uint8)
    ds = DeviceDataset(imgs, torch.arange(100), "cpu")
    def loader(rank, world):
        return DeviceLoader(ds, torch.zeros(8, 28, 28, 1), torch.zeros(8, dtype=torch.int32), rank=rank,
                            world=world, seed=3)
    l0, l1, ref = loader(0, 2), loader(1, 2), loader(0, 1)
    ref16 = DeviceLoader(ds, torch.zeros(16, 28, 28, 1), torch.zeros(16, dtype=torch.int32), seed=3)
    for _ in range(20):            # crosses several epochs of the 100-row dataset
        l0.next(); l1.next(); ref16.next()
        assert torch.equal(torch.cat([l0.out_labels, l1.out_labels]), ref16.out_labels)
    l2 = loader(1, 2)
    l2.seek(19)
    l1b = loader(1, 2)
    for _ in range(19):
        l1b.next()
    l2.next(); l1b.next()
    assert torch.equal(l2.out_labels, l1b.out_labels)

    # lookahead bookkeeping (the rows themselves are written on the GPU by the optimizer
    # launch, tests/test_fused_launch_gpu.py): no job off the resident-GPU mode; a recorded
    # position makes exactly the matching next() skip its gather, any other falls through
    assert l0.lookahead_job() is None
    la = loader(0, 1)
    la.next()
    la._ahead = la.pos                       # what lookahead_job records
    before = la.out_labels.clone()
    la.out_labels.fill_(-1)
    assert la.next() == 8 and la.pos == 16 and la._ahead is None
    assert int(la.out_labels.min()) == -1    # skipped: the optimizer launch wrote this batch
    la._ahead = 0                            # stale (e.g. after seek): gather as usual
    la.next()
    assert la.pos == 24 and int(la.out_labels.min()) >= 0 and not torch.equal(la.out_labels, before)


def test_meta_graph_def_structure(tmp_path):
    """model.ckpt-N.meta is a MetaGraphDef of the checkpoint's variable graph: one VariableV2
    (+ initializer / Assign / read) per saved tensor with its dtype and shape, the variables /
    trainable_variables / global_step collections of VariableDef records, the model
    description as JSON in MetaInfoDef.any_info; graph.pbtxt is the same graph as text.
    (Parity unpinned: no TensorFlow here to import it -- the structure is decoded by hand.)"""
    import numpy as np
    from distributed_tensorflow_ibm_mnist_amd.ckpt import metagraph as mg
    from distributed_tensorflow_ibm_mnist_amd.ckpt.saver import Saver, write_graph_pbtxt
    from distributed_tensorflow_ibm_mnist_amd.utils.proto import to_dict
    t = {"conv1/weights": np.zeros((5, 5, 1, 32), np.float32), "conv1/biases": np.ones(32, np.float32),
         "conv1/weights/ExponentialMovingAverage": np.zeros((5, 5, 1, 32), np.float32),
         "global_step": np.array(7, np.int64), "total_loss/avg": np.array(0.5, np.float32),
         "loader/epoch": np.array([3, 1], np.int32)}
    prefix = Saver().save(str(tmp_path), 7, t, meta={"model": "reference_cnn", "in_channels": 1})
    raw = open(prefix + ".meta", "rb").read()
    top = to_dict(raw)
    nodes = [to_dict(n) for n in to_dict(top[2][0])[1]]
    by_name = {n[1][0].decode(): n for n in nodes}
    assert len(nodes) == 4 * len(t)
    v = by_name["conv1/weights"]
    assert v[2][0] == b"VariableV2"
    attrs = {to_dict(a)[1][0].decode(): to_dict(to_dict(a)[2][0]) for a in v[5]}
    assert attrs["dtype"][6][0] == mg.DT_FLOAT
    dims = [to_dict(d)[1][0] for d in to_dict(attrs["shape"][7][0])[2]]
    assert dims == [5, 5, 1, 32]
    gs = {to_dict(a)[1][0].decode(): to_dict(to_dict(a)[2][0]) for a in by_name["global_step"][5]}
    assert gs["dtype"][6][0] == mg.DT_INT64 and 2 not in to_dict(gs["shape"][7][0])   # scalar
    assert [i.decode() for i in by_name["conv1/biases/Assign"][3]] == ["conv1/biases", "conv1/biases/Initializer/zeros"]
    # DT_INT32 initializer: TensorProto.int_val is field 7 (6 would be double_val)
    ia = {to_dict(a)[1][0].decode(): to_dict(to_dict(a)[2][0]) for a in by_name["loader/epoch/Initializer/zeros"][5]}
    tp = to_dict(ia["value"][8][0])
    assert tp[1][0] == mg.DT_INT32 and 7 in tp and 6 not in tp
    colls = {to_dict(c)[1][0].decode(): to_dict(c)[2][0] for c in top[4]}
    assert set(colls) == {"variables", "trainable_variables", "global_step"}

    def var_names(c):
        return [to_dict(d)[1][0].decode() for d in to_dict(to_dict(c)[2][0])[1]]
    assert sorted(var_names(colls["trainable_variables"])) == ["conv1/biases:0", "conv1/weights:0"]
    assert len(var_names(colls["variables"])) == len(t)
    assert mg.read_meta_json(prefix + ".meta")["in_channels"] == 1
    write_graph_pbtxt(str(tmp_path), t)
    txt = open(tmp_path / "graph.pbtxt").read()
    assert txt.count("node {") == 4 * len(t) and 'op: "VariableV2"' in txt and "producer: 134" in txt
    # a round-1/2 checkpoint's JSON .meta still reads
    old = tmp_path / "old.meta"
    old.write_text('{"model": "lenet5", "in_channels": 1}')
    assert mg.read_meta_json(str(old))["model"] == "lenet5"
