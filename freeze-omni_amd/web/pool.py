"""Stand-in for the absent web.pool module imported by bin/inference.py:27: re-exports bin.pool."""
from bin.pool import TTSObjectPool, pipelineObjectPool  # noqa: F401
