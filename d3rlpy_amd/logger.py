"""Offline metrics logger (the file layout of d3rlpy/logger.py:61-194, without
structlog / tensorboardX / wandb — no network access ever)."""
from __future__ import annotations

import json
import os
from datetime import datetime
from typing import Dict


class OfflineLogger:
    def __init__(self, experiment_name: str, save_metrics: bool = True,
                 root_dir: str = "d3rlpy_logs", verbose: bool = True,
                 with_timestamp: bool = True):
        self._save = save_metrics
        self._verbose = verbose
        name = experiment_name
        if with_timestamp:
            name += "_" + datetime.now().strftime("%Y%m%d%H%M%S%f")
        self.experiment_name = name
        self.logdir = os.path.join(root_dir, name)
        if save_metrics:
            os.makedirs(self.logdir, exist_ok=True)

    def add_epoch(self, epoch: int, step: int, metrics: Dict[str, float],
                  timings: Dict[str, float]) -> None:
        allm = dict(metrics)
        allm.update(timings)
        if self._save:
            for k, v in allm.items():
                with open(os.path.join(self.logdir, f"{k}.csv"), "a") as f:
                    print(f"{epoch},{step},{v}", file=f)
        if self._verbose:
            print(json.dumps({"epoch": epoch, "step": step, **allm}))

    def save_model(self, step: int, algo) -> None:
        if self._save:
            algo.save_model(os.path.join(self.logdir, f"model_{step}.pt"))

    def close(self) -> None:
        pass
