"""``MiningConfig.json`` - byte-compatible with the reference schema
(``miner/src/types.ts:3-54``, example ``miner/MiningConfig.example.json``).

Unknown keys (including the ``"//"`` comment keys) are ignored, exactly as the
reference does.  One optional extension block, ``"mi355x"``, configures this
node; the reference ignores it as an unknown key.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Dict, List, Literal, Optional

from pydantic import BaseModel, ConfigDict, Field, model_validator

# Task streams per GPU where a model's best differs from ``mi355x.workers_per_gpu`` (bench.py sweeps:
# profiles/bench_r4_stream_group_sweep.md).
DEFAULT_MODEL_STREAMS = {"anythingv3": 3, "kandinsky2": 2, "zeroscopev2xl": 2, "damo": 2, "robust_video_matting": 2}
# Lock-step group size where a model's best differs from ``mi355x.lockstep_group``.  anythingv3: 3 streams x
# groups of 8 (batch 16 on the batch-8 canonical plans, with tile families tuned for the batch-16 shapes at
# the pinned splits - bitwise neutral) measured +2.2 % over 4 x 4 on one box (profiles/sd_groups_r5.md).
# kandinsky2: 2 streams x groups of 8 with its batch-16 families, +1.8 % over 4 x 4 at the same p50 latency
# and 3.3 instead of 5.3 host cores (profiles/r6/k2/).
DEFAULT_MODEL_LOCKSTEP = {"anythingv3": 8, "kandinsky2": 8}


class _Base(BaseModel):
    model_config = ConfigDict(extra="ignore", populate_by_name=True)


class BlockchainConfig(_Base):
    private_key: str = ""
    rpc_url: str = ""
    use_delegated_validator: bool = False
    delegated_validator_address: str = ""


class RPCConfig(_Base):
    host: str = "localhost"
    port: int = 8335


class AutomineConfig(_Base):
    enabled: bool = False
    delay: int = 60
    version: int = 0
    model: str = ""
    fee: str = "0"
    input: dict = Field(default_factory=dict)


class CogEntry(_Base):
    url: str = ""


class ReplicateConfig(_Base):
    api_token: Optional[str] = None


class MLConfig(_Base):
    strategy: Literal["cog", "replicate", "local"] = "local"
    cog: Dict[str, CogEntry] = Field(default_factory=dict)
    replicate: ReplicateConfig = Field(default_factory=ReplicateConfig)

    @model_validator(mode="before")
    @classmethod
    def _drop_comments(cls, v):
        if isinstance(v, dict) and isinstance(v.get("cog"), dict):
            v = dict(v)
            v["cog"] = {k: e for k, e in v["cog"].items() if k != "//" and isinstance(e, dict)}
        return v


class HttpClientConfig(_Base):
    url: str = "http://127.0.0.1:5001"


class PinataConfig(_Base):
    jwt: str = ""


class IPFSConfig(_Base):
    strategy: Literal["http_client", "pinata", "local"] = "local"
    http_client: HttpClientConfig = Field(default_factory=HttpClientConfig)
    pinata: PinataConfig = Field(default_factory=PinataConfig)


class MI355XConfig(_Base):
    """Extension block (ignored by the reference miner)."""
    gpus: Optional[int] = None            # default: all visible
    models: List[str] = Field(default_factory=lambda: ["kandinsky2"])  # enabled model names
    model_ids: Dict[str, str] = Field(default_factory=dict)  # template name -> on-chain model id
    weights_dir: Optional[str] = None     # safetensors (+ tokenizer files); None = random-init (benchmark only)
    hang_timeout_s: float = 300.0         # kill a GPU worker whose busy slot has not progressed this long
    # one worker PROCESS per GPU even on a one-GPU node (the multi-GPU pool: watchdog respawn, a
    # one-rank RCCL communicator carrying the weight broadcast); default: in-process pool at 1 GPU
    worker_processes: bool = False
    # models.ts:185-194 quirks Q2/Q3 (decimal must be integral, max never enforced).  ON by default:
    # validity decides contestations, so this node must judge inputs as the deployed miners do
    reference_hydration_quirks: bool = True
    job_lease_seconds: float = 900.0
    poll_interval_ms: int = 100           # index.ts:1081
    log_window_blocks: int = 2000         # eth_getLogs back-fill window (halved on provider errors)
    min_model_filter_fee: str = "0"      # MiningFilter.minfee of every enabled model (wei)
    verify_fraction: float = 0.0          # re-solve this fraction of others' solutions (Q10)
    chain_id: Optional[int] = None
    mock_chain: bool = False              # in-process MockEngine (testing / plumbing config)
    selftest: bool = True                 # boot CID self-test (index.ts:981-1001)
    selftest_table: Optional[str] = None  # override of config/selftest.json
    workers_per_gpu: int = 4              # task slots per GPU (pipeline forks), capped per model by
                                          # model_streams (anythingv3 3, kandinsky2 2); 1 = latency mode
    # per-model cap on those streams.  Kandinsky2, measured on one box with every task stream on its own
    # hardware queue (round 6, batch-16 families, profiles/r6/k2/): 7,860-7,902 tasks/h at 2 streams x
    # groups of 8, 7,697-7,799 at 4 x 4, 7,836-7,959 at 3 x 8 (p50 +48 %), 7,790 at 4 x 8, 7,398 at 5 x 4.
    # The video UNet's activations fill the GPU at 2 streams (zeroscope 3 streams: 1,129).
    model_streams: Dict[str, int] = Field(default_factory=lambda: dict(DEFAULT_MODEL_STREAMS))
    # IPFS gateway (http(s) base URL) for the input of a task whose transaction is not a plain
    # submitTask call (submitted through a contract): the bytes are fetched by the
    # task's on-chain CID and accepted only if their on-chain CIDv0 matches.  None: $ARBIUS_IPFS_GATEWAY,
    # else only the configured pinner (kubo cat / the local store) is asked.
    ipfs_gateway: Optional[str] = None
    # task -> GPU policy of the multi-GPU pool (parallel/dispatch.py): "spread" = least-loaded GPU
    # first (lowest latency below saturation, profiles/dispatch_r5.md), "pack" = fill one GPU first
    dispatch_policy: Literal["spread", "pack"] = "spread"
    lockstep_group: int = 4               # queued compatible SD tasks solved per stream in ONE batch
                                          # (batch-invariant plans: same CIDs as solo; a lone task
                                          # never waits for company)
    model_lockstep: Dict[str, int] = Field(default_factory=lambda: dict(DEFAULT_MODEL_LOCKSTEP))
    # node-rate control plane (node/miner.py, chain/rpc.py, chain/txpipe.py)
    job_concurrency: Dict[str, int] = Field(default_factory=dict)   # per job method, over miner.JOB_LIMITS
    event_poll_ms: int = 1000             # eth_getLogs poll period (its own loop, never behind jobs)
    event_concurrency: int = 64           # tasks whose events are handled at once within a poll window
    rpc_batch: bool = True                # JSON-RPC batches for reads issued together (off: one POST each)
    rpc_max_batch: int = 50               # calls per batch POST (provider limits)
    tx_stuck_s: float = 12.0              # re-broadcast / fee-bump the lowest unmined nonce after this
    # host-CPU admission (parallel/cpu_budget.py): a model whose per-GPU core budget does not fit every GPU
    # (robust_video_matting with host H.264 encode: 13.4 cores per GPU) runs on fewer workers;
    # host_cores overrides sched_getaffinity
    cpu_admission: bool = True
    host_cores: Optional[int] = None


class MiningConfig(_Base):
    log_path: Optional[str] = None
    db_path: str = "db.sqlite"
    stake_buffer_percent: float = 20
    stake_buffer_topup_percent: float = 1
    evilmode: bool = False
    blockchain: BlockchainConfig = Field(default_factory=BlockchainConfig)
    rpc: RPCConfig = Field(default_factory=RPCConfig)
    automine: AutomineConfig = Field(default_factory=AutomineConfig)
    ml: MLConfig = Field(default_factory=MLConfig)
    ipfs: IPFSConfig = Field(default_factory=IPFSConfig)
    mi355x: MI355XConfig = Field(default_factory=MI355XConfig)

    @model_validator(mode="after")
    def _check(self):
        # reference defect Q14 (blockchain.ts:31-35): delegated validator leaves `solver`
        # undefined -> reject at load instead of failing later.
        if self.blockchain.use_delegated_validator:
            raise ValueError("use_delegated_validator is not supported (reference leaves solver undefined)")
        return self

    @staticmethod
    def load(path: str) -> "MiningConfig":
        return MiningConfig.model_validate(json.loads(Path(path).read_text()))

    @staticmethod
    def from_dict(d: dict) -> "MiningConfig":
        return MiningConfig.model_validate(d)
