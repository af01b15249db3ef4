"""Stat logger with the reference's interface (src/utils/logging.py): `Logger(console_logger)`,
`log_stat(key, value, t, to_sacred=True)`, `print_recent_stats()`, `setup_tb(dir)`, `setup_sacred(run_dict)`,
the `stats` history ({key: [(t, value), ...]}) and `get_logger()`.

Every stat is kept in memory and fanned out to the optional sinks (tensorboard_logger, a sacred run's info dict),
which are attached the same way the reference attaches them. The learner logs plain Python floats (the HIP
learner's stats are read back once per logged step), so no sink ever sees a device tensor.
"""
import logging
from collections import defaultdict

import numpy as np

# the recent-stats window per key (epsilon is a schedule value: its last sample is the current one)
_WINDOW = {"epsilon": 1}
_DEFAULT_WINDOW = 5
_PER_LINE = 4


class Logger:
    def __init__(self, console_logger):
        self.console_logger = console_logger
        self.stats = defaultdict(list)
        self._sinks = {}          # name -> callable(key, value, t, to_sacred)

    # the reference's flags, derived from the attached sinks
    use_tb = property(lambda self: "tb" in self._sinks)
    use_sacred = property(lambda self: "sacred" in self._sinks)
    use_hdf = property(lambda self: False)

    def setup_tb(self, directory_name):
        from tensorboard_logger import configure, log_value   # optional dependency, as in the reference
        configure(directory_name)
        self._sinks["tb"] = lambda key, value, t, _: log_value(key, value, t)

    def setup_sacred(self, sacred_run_dict):
        info = sacred_run_dict.info

        def to_info(key, value, t, to_sacred):
            if to_sacred:
                info.setdefault("{}_T".format(key), []).append(t)
                info.setdefault(key, []).append(value)
        self.sacred_info = info
        self._sinks["sacred"] = to_info

    def log_stat(self, key, value, t, to_sacred=True):
        self.stats[key].append((t, value))
        for sink in self._sinks.values():
            sink(key, value, t, to_sacred)

    def recent(self, key):
        """Mean of the key's last few logged values (the figure print_recent_stats shows)."""
        hist = self.stats[key][-_WINDOW.get(key, _DEFAULT_WINDOW):]
        return float(np.mean([float(v) for _, v in hist]))

    def print_recent_stats(self):
        t_env, episode = self.stats["episode"][-1]
        cells = ["{:<25}{:>8}".format(k + ":", "{:.4f}".format(self.recent(k)))
                 for k in sorted(self.stats) if k != "episode"]
        rows = ["\t".join(cells[i:i + _PER_LINE]) for i in range(0, len(cells), _PER_LINE)]
        header = "Recent Stats | t_env: {:>10} | Episode: {:>8}\n".format(t_env, episode)
        self.console_logger.info(header + "\n".join(rows) + ("\n" if len(cells) % _PER_LINE == 0 and cells else ""))


def get_logger():
    """Root logger with one console handler ("[LEVEL hh:mm:ss] name message"), level DEBUG."""
    logger = logging.getLogger()
    handler = logging.StreamHandler()
    handler.setFormatter(logging.Formatter("[%(levelname)s %(asctime)s] %(name)s %(message)s", "%H:%M:%S"))
    logger.handlers = [handler]
    logger.setLevel("DEBUG")
    return logger
