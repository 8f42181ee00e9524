"""Op layer over the CDNA4 HIP kernels.

* ``functional`` -- shape-aware wrappers (explicit buffers, hipGraph-safe); used
  by the fused executor (``runtime/executor.py``).
* ``autograd``   -- ``torch.autograd.Function`` per op (conv, fused conv+ReLU+pool,
  dense, max-pool, LRN, softmax-CE).
* ``nn``         -- ``nn.Module`` layers and ``HipModel(spec)``: any registry model
  as a trainable ``nn.Sequential`` for stock PyTorch training loops.
"""
