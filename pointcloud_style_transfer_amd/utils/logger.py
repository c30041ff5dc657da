"""Console + file logger with the reference's constructor (`utils/logger.py:6-47`)."""
import logging
import os
import sys
from datetime import datetime


class Logger:
    def __init__(self, name: str, log_dir: str, experiment_name: str, file_output: bool = True):
        self.logger = logging.getLogger(name)
        self.logger.setLevel(logging.INFO)
        if self.logger.hasHandlers():
            self.logger.handlers.clear()
        fmt = logging.Formatter("%(asctime)s [%(levelname)s] [%(name)s]: %(message)s")
        ch = logging.StreamHandler(sys.stdout)
        ch.setFormatter(fmt)
        self.logger.addHandler(ch)
        if file_output:
            d = os.path.join(log_dir, experiment_name)
            os.makedirs(d, exist_ok=True)
            fh = logging.FileHandler(os.path.join(d, datetime.now().strftime("%Y%m%d_%H%M%S") + ".log"))
            fh.setFormatter(fmt)
            self.logger.addHandler(fh)

    def info(self, msg: str):
        self.logger.info(msg)

    def warning(self, msg: str):
        self.logger.warning(msg)

    def error(self, msg: str):
        self.logger.error(msg)
