"""Learner-facing Logger (reference: src/utils/logging.py:5-64): log_stat fan-out and recent-stat printing.
Tensorboard / sacred sinks are optional and enabled the same way as in the reference."""
import logging
from collections import defaultdict

import numpy as np


class Logger:
    def __init__(self, console_logger):
        self.console_logger = console_logger
        self.use_tb = False
        self.use_sacred = False
        self.use_hdf = False
        self.stats = defaultdict(lambda: [])

    def setup_tb(self, directory_name):
        from tensorboard_logger import configure, log_value
        configure(directory_name)
        self.tb_logger = log_value
        self.use_tb = True

    def setup_sacred(self, sacred_run_dict):
        self.sacred_info = sacred_run_dict.info
        self.use_sacred = True

    def log_stat(self, key, value, t, to_sacred=True):
        self.stats[key].append((t, value))
        if self.use_tb:
            self.tb_logger(key, value, t)
        if self.use_sacred and to_sacred:
            self.sacred_info.setdefault("{}_T".format(key), []).append(t)
            self.sacred_info.setdefault(key, []).append(value)

    def print_recent_stats(self):
        log_str = "Recent Stats | t_env: {:>10} | Episode: {:>8}\n".format(*self.stats["episode"][-1])
        i = 0
        for (k, v) in sorted(self.stats.items()):
            if k == "episode":
                continue
            i += 1
            window = 5 if k != "epsilon" else 1
            item = "{:.4f}".format(np.mean([float(x[1]) for x in self.stats[k][-window:]]))
            log_str += "{:<25}{:>8}".format(k + ":", item)
            log_str += "\n" if i % 4 == 0 else "\t"
        self.console_logger.info(log_str)


def get_logger():
    logger = logging.getLogger()
    logger.handlers = []
    ch = logging.StreamHandler()
    ch.setFormatter(logging.Formatter("[%(levelname)s %(asctime)s] %(name)s %(message)s", "%H:%M:%S"))
    logger.addHandler(ch)
    logger.setLevel("DEBUG")
    return logger
