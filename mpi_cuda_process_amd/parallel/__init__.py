"""Parallelism: slab decomposition, process bootstrap and halo transports.

* :mod:`.decomp` — 1-D slab split along the slowest axis (z; rows in 2D) with uneven remainder.
* :mod:`.dist`   — one-process-per-GPU bootstrap over ``torch.distributed`` (torchrun / mpirun env),
  RCCL unique-id distribution, and the ``torch`` callback transport (point-to-point isend/irecv
  through any process group: gloo on CPU, nccl = RCCL on GPU).

Reference parity: the reference's only parallelism is a hard-wired 2-rank row split with MPI
point-to-point halo rows (MDF_kernel.cu:30,38,54,62,167-183). Here P is any number <= nz.
"""

from .decomp import owner, slab_bounds  # noqa: F401
from .dist import (DistEnv, TorchP2PTransport, broadcast_bytes, detect_env,  # noqa: F401
                   init_distributed, is_distributed)
