import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, "sofa-jraft_amd"); sys.path.insert(0, "oracle")
import numpy as np
import jraft_oracle as oracle
from jraft_amd import Engine, Table
from quorum_cases import random_batch
from test_gpu_table import states_of, match_recs, committed_from
with Engine(0) as e:
    for P, G, rp in ((1, 64, 0.4), (1, 64, 0.0), (2, 64, 0.4), (1, 4096, 0.4), (3, 64, 0.4)):
        b = random_batch(1000 + P, G, P, run_prob=rp)
        ce, se, _ = oracle.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"], b["last_committed"], b["conf"], b["run_off"], b["run_start"], b["run_conf"], chunk=7)
        t = Table(e, G, P)
        t.update(states_of(b), match_recs(b["match"], b["pending_index"]))
        changed, st = t.epoch(status=True)
        bad = np.nonzero(st != se)[0]
        ro = b["run_off"]
        fl = [g for g in range(G) if ro[g+1]-ro[g] > 1]
        print(P, G, rp, "bad", bad[:20].tolist(), "nbad", len(bad), "nonzero want", np.nonzero(se)[0][:20].tolist(), "flagged", fl[:12])
        t.close()
