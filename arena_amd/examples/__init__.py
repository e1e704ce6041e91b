"""Bundled reference workloads (the demos the reference's docs run inside its images).

* ``mnist``      -- standalone / allreduce MNIST MLP (mnist_with_summaries equivalent; fused HIP
                    kernels + hipGraphs on MI355X, reference ops on CPU).
* ``mnist_ps``   -- PS/worker MNIST (TF dist-mnist equivalent) over the native parameter server.
* ``mnist_hvd``  -- the same model as a plain ``torch.nn`` module trained with the Horovod-style
                    ``arena_amd.parallel.hvd`` API (generic DistributedOptimizer path).
"""
