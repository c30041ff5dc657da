"""Console + file logger with the reference's constructor and methods (`utils/logger.py:6-47`):
records go to stdout and, with `file_output`, to `<log_dir>/<experiment_name>/<YYYYmmdd_HHMMSS>.log`,
formatted "time [LEVEL] [name]: message"; constructing a logger again replaces its handlers."""
import logging
import os
import sys
import time

_FORMAT = "%(asctime)s [%(levelname)s] [%(name)s]: %(message)s"


def _sinks(log_dir: str, experiment_name: str, file_output: bool):
    yield logging.StreamHandler(sys.stdout)
    if file_output:
        folder = os.path.join(log_dir, experiment_name)
        os.makedirs(folder, exist_ok=True)
        yield logging.FileHandler(os.path.join(folder, time.strftime("%Y%m%d_%H%M%S") + ".log"))


class Logger:
    def __init__(self, name: str, log_dir: str, experiment_name: str, file_output: bool = True):
        log = logging.getLogger(name)
        log.setLevel(logging.INFO)
        log.handlers.clear()
        formatter = logging.Formatter(_FORMAT)
        for sink in _sinks(log_dir, experiment_name, file_output):
            sink.setFormatter(formatter)
            log.addHandler(sink)
        self.logger = log
        # the reference's three methods, bound straight to the logging calls
        self.info, self.warning, self.error = log.info, log.warning, log.error
