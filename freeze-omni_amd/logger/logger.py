"""Stand-in for the absent logger.logger module (models/pipeline.py:7): stdlib logging."""
import logging


def setup_logger(name, file_log_level="DEBUG", terminal_log_level="INFO"):
    log = logging.getLogger(name)
    if not log.handlers:
        h = logging.StreamHandler()
        h.setLevel(getattr(logging, terminal_log_level, logging.INFO))
        h.setFormatter(logging.Formatter("%(asctime)s %(name)s %(levelname)s %(message)s"))
        log.addHandler(h)
    log.setLevel(getattr(logging, file_log_level, logging.DEBUG))
    return log
