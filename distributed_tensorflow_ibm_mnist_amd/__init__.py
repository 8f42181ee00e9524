"""MI355X-native distributed MNIST trainer with the capabilities of
``cybera/distributed_tensorflow_ibm_mnist``.

Layers (mirrors SURVEY.md §1, re-designed for MI355X):

* ``utils``     flags (tf.app.flags surface), parameter manager (tf_parameter_mgr)
* ``data``      IDX / PNG / TFRecord / synthetic sources, device-resident loader
* ``models``    reference CNN (mnist_input.inference), LeNet-5, MLP; torch oracles
* ``ops``       HIP/CDNA4 kernels (MFMA GEMM/conv, pool, LRN, softmax-CE, fused
                optimizer) behind thin Python wrappers; autograd Functions
* ``runtime``   static execution plan + arena buffers + hipGraph capture
* ``parallel``  RCCL data parallel (bucketed, overlapped) and parameter-server mode
* ``train``     MonitoredTrainingSession equivalent, hooks, trainer
* ``ckpt``      TF tensor-bundle checkpoint writer/reader (same layout/names)
* ``obs``       tfevents writer, DLMAO-equivalent Monitor, timers
"""

__version__ = "0.1.0"
