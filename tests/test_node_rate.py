"""The node sustains an 8-GPU task rate on a latent chain.

``node/chainsim.py``: MockNode in its own process with 250 ms blocks, a mempool and 30 ms per
JSON-RPC request; the real ``Miner`` + ``RpcChainClient`` (batched reads, pipelined sender); a
``FakeSolverPool`` at 8 GPUs x 8.8 tasks/s (192 solve servers of 2.73 s); chain time 200x wall
time, so the 2,120 s claim delay elapses at 10.6 s and claims fall due at the solve rate for the
rest of the run (6,000 simulated seconds); one accepted transaction is dropped by the sequencer.
Round 5's scheduler and sender completed 17 of 2,112 offered tasks under the same harness
(``profiles/node_rate_r6.md``).
"""
import math

from arbius_amd.node.chainsim import run_chain_sim


def test_node_sustains_8_gpu_rate_with_claims_due_and_a_dropped_tx(tmp_path):
    r = run_chain_sim(gpus=8, rate_per_gpu=8.8, latency_s=0.03, block_time_s=0.25, accel=200.0, load_s=30.0,
                      drop_at_s=12.0, stuck_s=4.0, workdir=str(tmp_path))
    assert r["simulated_s"] >= 3000
    assert not math.isnan(r["completed_rate"]) and r["completed_frac"] >= 0.95, r
    assert r["solutions"] == r["offered_tasks"], r          # every offered task solved on chain
    assert r["claimed"] == r["solutions"], r                 # and every claim landed
    assert r["max_poll_gap_s"] <= 2.0, r
    assert len(r["dropped_txs"]) == 1 and r["txpipe"]["rebroadcasts"] >= 1, r   # the dropped tx recovered
    assert r["mempool_left"] == 0 and r["txpipe"]["replaced"] == 0, r          # no nonce gap left behind
    assert not r["jobs_failed"], r
