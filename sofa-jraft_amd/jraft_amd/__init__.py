"""jraft_amd -- Python face of the MI355X-native SOFAJRaft quorum + CRC64 engine.

The product is libjrq.so (sofa-jraft_amd/csrc, ABI in include/jrq.h); this
package binds it with ctypes and provides the seeded synthetic workloads used
by tests and bench.py.
"""
from ._lib import (CONF_RUNS, ST_EMPTY_CONF, ST_NOT_LEADER, ST_OK, ST_OUT_OF_RANGE, JrqError,
                   conf_word, load)
from .engine import Engine, Table, decode_changed

__all__ = ["Engine", "JrqError", "conf_word", "load", "ST_OK", "ST_NOT_LEADER",
           "ST_OUT_OF_RANGE", "ST_EMPTY_CONF", "CONF_RUNS", "Table", "decode_changed"]
