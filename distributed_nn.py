"""Training entry point (same name and flags as the reference's ``src/distributed_nn.py``).

    torchrun --standalone --nproc-per-node 8 distributed_nn.py --network VGG11 --dataset Cifar10 \
        --batch-size 64 --momentum 0.9 --method 5 --max-steps 1000

One process per GPU (RCCL over xGMI); ``RANK``/``WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT`` come from
the launcher exactly as in the reference (``distributed_nn.py:75-78``).  Without ``--data-dir`` the
dataset is synthetic data of the real dataset's shape.
"""
import sys

import ewdml
from ewdml.runtime import run


def main(argv=None):
    cfg = ewdml.parse_args(argv)
    res = run(cfg)
    return res


if __name__ == "__main__":
    main(sys.argv[1:])
