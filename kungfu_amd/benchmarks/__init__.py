"""All-reduce micro-benchmark over real model gradient sizes.

``python -m kungfu_amd.benchmarks --method CPU|RCCL|RCCL+CPU|HIER --model resnet50``
(parity: ``python -m kungfu.tensorflow.v1.benchmarks --method CPU|NCCL|NCCL+CPU|HOROVOD``,
``srcs/python/kungfu/tensorflow/v1/benchmarks/__main__.py:135-188``).  Reports
the reference's "equivalent data rate" tot_size*4(np-1)/t in GiB/s and a
``RESULT: mean +-1.96sigma`` line.
"""
