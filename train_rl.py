"""Trainer entry point with the reference's name and flags (train_rl.py:292-787):

    python train_rl.py --config configs/training/16x16x40_medium.yaml --updates 500 --out runs/x
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train_rl.py --config ...

Runs ms_amd.train.main (one process per GPU; RCCL gradient all-reduce when WORLD_SIZE > 1)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "minesweeper-ppo_amd"))

from ms_amd.train import main  # noqa: E402

if __name__ == "__main__":
    main()
