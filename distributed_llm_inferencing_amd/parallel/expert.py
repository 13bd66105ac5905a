"""Expert parallelism for Mixtral: experts mapped to GPU ranks, all-to-all over xGMI
(BASELINE.json config 5; SURVEY.md §2.4 C4, §2.5 "Expert parallel"; the reference has no
MoE at all — its compute is HF ``generate`` at ``worker/app.py:297-305``).

Layout: data-parallel attention + expert-parallel MoE. Every rank holds the full attention
/ norm / embedding weights and its own requests + paged KV; rank r holds experts
[r*E/N, (r+1)*E/N). Per MoE layer, all on device:

    route (gate logits -> softmax -> top-2 -> renormalise)   moe_router kernel
    dispatch pack: (token, pick) rows into per-rank buckets  ep_pack kernel
    all_to_all_single (rows + their expert ids)              RCCL, all 7 xGMI links at once
    local expert MLPs on the rows received                   moe_align/gather + grouped GEMM
    all_to_all_single back, weighted sum per token           moe_combine kernel

Decode steps use FIXED-CAPACITY buckets: a token's top-k experts are distinct, so a rank
sends at most min(k, E/N) rows per token to any peer; with every rank's token count T_p of
the step known, bucket sizes are exact bounds (no dropped tokens, identical results) and
nothing about the routing is read on the host. The T_p come from the ONE per-step lockstep
exchange every rank makes anyway (do we still have work? how many tokens?): O(1) host syncs
per decode step, none per layer. Prefill steps (T in the thousands) would move mostly
padding at that bound, so they exchange exact per-destination counts per layer (one host
read per layer; prefill is compute-bound).

Ranks step in lockstep: every rank launches one forward per step (a rank without work runs
an empty one that still joins every exchange); lookahead scheduling stays on (a rank's
next step is planned against its in-flight one before the lockstep exchange).
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import ops
from ..engine.batch import DECODE
from ..engine.llm_engine import LLMEngine
from ..models.configs import get_config
from ..models.model import TransformerLM
from ..models import weights as W

# a step whose largest per-rank token count exceeds this exchanges exact counts per layer
EP_BOUND_MAX_TOKENS = int(os.environ.get("DLI_EP_BOUND_MAX_TOKENS", "1024"))
_log = logging.getLogger("dli.expert")


class ExpertParallelMoE:
    """Installed as ``TransformerLM.moe_fn`` on every rank.

    Two data planes. ``torch``: three ``all_to_all_single`` per layer over fixed-capacity
    buckets (below). ``ipc`` (``DLI_EP_COMM=ipc``): the mailbox transport
    (``csrc/runtime/ipc.cpp`` ``dli_ipc_ep``; on CPU its host model in ``fifo.py``). The
    per-destination row counts produced by ``ep_pack`` stay on the device and travel in each
    message's header; the copy kernels move exactly the routed rows (no padding on the
    wire) into the peer's mailbox, and the peer's expert rows come back the same way. No
    host value is needed per layer, so the decode forward (attention + every MoE exchange)
    is captured in one hipGraph per batch bucket; the only host sync per step is the
    lockstep exchange."""

    def __init__(self, num_experts: int, top_k: int, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if num_experts % self.world:
            raise ValueError(f"{num_experts} experts do not split over {self.world} ranks")
        self.E, self.k = num_experts, top_k
        self.e_per = num_experts // self.world
        self.e0 = self.rank * self.e_per
        self.per_token = min(top_k, self.e_per)        # rows per token to any one rank
        self.bytes_sent = 0
        self.exchanges = 0
        self.host_reads = 0                            # routing-dependent host syncs
        self.peer_tokens: Optional[List[int]] = None   # T of every rank for this step
        self._bases = {}
        self.ep = None                 # mailbox endpoint (setup_ipc)
        self.static = False            # capturing / replaying graphs: fixed region sizes
        self.graph_tokens = 0          # largest decode batch per rank (graph regions)
        self.rows_sent = 0             # rows this rank sent to other ranks (dispatch)
        self.rows_routed = 0           # routed (token, pick) rows produced on this rank

    def expert_range(self):
        return (self.e0, self.e0 + self.e_per)

    def setup_ipc(self, device, dim: int, dtype, max_tokens: int, graph_tokens: int) -> None:
        """Mailboxes for every ordered pair of ranks, each holding one layer's worth of rows
        from a step of up to ``max_tokens`` tokens (``min(k, E/N)`` rows per token)."""
        from .fifo import ShmMailboxTransport
        N, me = self.world, self.rank
        self.row_bytes = dim * torch.empty(0, dtype=dtype).element_size()
        self.cap = max_tokens * self.per_token
        self.graph_tokens = graph_tokens
        dev = torch.device(device)
        if dev.type == "cuda":
            from ..runtime import IpcEndpoint
            eb = IpcEndpoint.ep_bytes(self.cap, self.row_bytes)
        else:
            eb = 8 + 8 + self.cap * 4 + self.cap * self.row_bytes + 64
        cap = [[0 if s == d else eb for d in range(N)] for s in range(N)]
        box = [f"/dli_ep_{os.environ.get('MASTER_PORT', '0')}_{os.getpid()}"
               if me == 0 else None]
        dist.broadcast_object_list(box, src=0, group=self.group)
        if dev.type == "cuda":
            from ..runtime import IpcEndpoint
            ep = IpcEndpoint(N, me, cap)
            hs = [None] * N
            dist.all_gather_object(hs, ep.handles(), group=self.group)
            dist.barrier(group=self.group)
            ep.connect(hs)
        else:
            ep = ShmMailboxTransport(N, me, cap, box[0])
            dist.barrier(group=self.group)
            ep.connect()
        dist.barrier(group=self.group)
        self.ep = ep
        self.caps = [self.cap] * N

    def close(self) -> None:
        if self.ep is not None:
            self.ep.close()
            self.ep = None

    def _call_ipc(self, h, topk_w, topk_ids, lp) -> torch.Tensor:
        T, D = h.shape
        dev = h.device
        N, me, pt = self.world, self.rank, self.per_token
        C = T * pt                                   # my rows for one destination, at most
        send_base = [p * C for p in range(N)]
        key = (C, str(dev))
        base = self._bases.get(key)
        if base is None:
            base = torch.tensor(send_base, dtype=torch.int32, device=dev)
            self._bases[key] = base
        # receive region of source q: a peer replaying a decode graph routes EVERY row of its
        # padded bucket (up to graph_tokens rows, not its announced token count), so an eager
        # rank (idle, or running a small prefill) reserves at least the largest bucket for it
        if self.static:          # a captured graph: regions sized for any decode batch
            rcap = [self.graph_tokens * pt] * N
        else:
            rcap = [max(t, self.graph_tokens) * pt for t in self.peer_tokens]
        recv_base = [0] * N
        for q in range(1, N):
            recv_base[q] = recv_base[q - 1] + rcap[q - 1]
        R = sum(rcap)
        send_x, send_e, pos, cnt = ops.ep_pack(h, topk_ids, self.e_per, base, N * C,
                                               counts=True)
        if send_x.shape[0] == 0:                     # an idle rank still joins
            send_x = h.new_zeros(1, D)
            send_e = torch.full((1,), -1, dtype=torch.int32, device=dev)
        recv_x = h.new_empty(max(R, 1), D)
        recv_e = torch.empty(max(R, 1), dtype=torch.int32, device=dev)
        recv_cnt = torch.zeros(N, dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0
        self.ep.ep(st, False, self.row_bytes, send_x, send_e, send_base, cnt, recv_x, recv_e,
                   recv_base, rcap, recv_cnt, self.caps, self.caps, send_cap=C)
        if R > 0:
            y = ops.moe_mlp(recv_x[:R], lp["w_gu"], lp["w_down"],
                            torch.ones(R, 1, dtype=torch.float32, device=dev),
                            recv_e[:R].view(R, 1), self.e0, plan_rows=self._plan_rows())
        else:
            y = recv_x
        self.ep.ep(st, True, self.row_bytes, send_x, send_e, send_base, cnt, y, None,
                   recv_base, rcap, recv_cnt, self.caps, self.caps, send_cap=C)
        self.exchanges += 1
        self.rows_routed += T * self.k
        if dev.type != "cuda":           # host model: counts are readable for the tests
            self.rows_sent += int(cnt.sum()) - int(cnt[me])
        if T == 0:
            return h.new_zeros(0, D)
        return ops.moe_combine(send_x, topk_w, pos)

    def _plan_rows(self) -> int:
        """Routed rows this rank's experts receive on average for the step's token counts:
        every rank's tokens x top-k, spread over the N ranks' experts. The receive region is
        sized for the worst case; the grouped-GEMM plan is the one autotuned for this
        (``StageRunner.autotune``: bucket x top-k rows over the local experts)."""
        return max(1, sum(self.peer_tokens) * self.k // self.world)

    def begin_step(self, peer_tokens: List[int]) -> None:
        """Every rank's token count for the forward about to run (same list everywhere)."""
        self.peer_tokens = [int(t) for t in peer_tokens]

    def _cdev(self, dev):
        return dev if dist.get_backend(self.group) == "nccl" else torch.device("cpu")

    def _a2a(self, out, inp, out_splits, in_splits):
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def __call__(self, h: torch.Tensor, lp: dict, layer: int, routing=None) -> torch.Tensor:
        T, D = h.shape
        dev = h.device
        k, N = self.k, self.world
        if self.peer_tokens is None or len(self.peer_tokens) != N or \
                self.peer_tokens[self.rank] != T:
            raise RuntimeError("ExpertParallelMoE: begin_step() must announce this step's "
                               "token counts before the forward")
        if T > 0:
            topk_w, topk_ids = (routing if routing is not None
                                else ops.moe_router(h, lp["router"], k))
        else:
            topk_w = torch.zeros(0, k, dtype=torch.float32, device=dev)
            topk_ids = torch.zeros(0, k, dtype=torch.int32, device=dev)
        if self.ep is not None:
            return self._call_ipc(h, topk_w, topk_ids, lp)
        bound = max(self.peer_tokens) <= EP_BOUND_MAX_TOKENS
        if bound:
            # fixed-capacity buckets: C_p = T_p * min(k, E/N) rows from rank p to each rank
            C = T * self.per_token
            in_splits = [C] * N
            out_splits = [t * self.per_token for t in self.peer_tokens]
            key = (C, str(dev))
            base = self._bases.get(key)
            if base is None:
                base = torch.arange(N, dtype=torch.int32, device=dev) * C
                self._bases[key] = base
        else:
            # exact per-destination counts (prefill): one host read per layer
            if T > 0:
                dest = topk_ids.reshape(-1).long() // self.e_per
                sc = torch.bincount(dest, minlength=N).to(torch.int32)
            else:
                sc = torch.zeros(N, dtype=torch.int32, device=dev)
            cd = self._cdev(dev)
            rc = torch.empty(N, dtype=torch.int32, device=cd)
            dist.all_to_all_single(rc, sc.to(cd), group=self.group)
            both = torch.cat([sc.to(cd), rc]).tolist()
            self.host_reads += 1
            in_splits, out_splits = both[:N], both[N:]
            base = torch.zeros(N, dtype=torch.int32, device=dev)
            if N > 1:
                base[1:] = torch.cumsum(sc, 0)[:-1].to(torch.int32)
        send_rows, recv_rows = sum(in_splits), sum(out_splits)
        send_x, send_e, pos = ops.ep_pack(h, topk_ids, self.e_per, base, send_rows)
        cd = self._cdev(dev)
        recv_x = torch.empty(recv_rows, D, dtype=h.dtype, device=cd)
        recv_e = torch.empty(recv_rows, dtype=torch.int32, device=cd)
        self._a2a(recv_x, send_x.to(cd), out_splits, in_splits)
        self._a2a(recv_e, send_e.to(cd), out_splits, in_splits)
        recv_x, recv_e = recv_x.to(dev), recv_e.to(dev)
        # local experts: one expert per received row (weight 1); padding rows (id -1) fall
        # outside the local range, are skipped by the align and come back as zeros
        if recv_rows > 0:
            y = ops.moe_mlp(recv_x, lp["w_gu"], lp["w_down"],
                            torch.ones(recv_rows, 1, dtype=torch.float32, device=dev),
                            recv_e.view(recv_rows, 1), self.e0, plan_rows=self._plan_rows())
        else:
            y = recv_x.new_zeros(0, D)
        back = torch.empty(send_rows, D, dtype=h.dtype, device=cd)
        self._a2a(back, y.to(cd), in_splits, out_splits)
        back = back.to(dev)
        self.exchanges += 1
        self.bytes_sent += (send_rows + recv_rows) * D * h.element_size()
        if T == 0:
            return h.new_zeros(0, D)
        return ops.moe_combine(back, topk_w, pos)


class ExpertParallelEngine:
    """One rank of a DP-attention / EP-MoE Mixtral deployment (all ranks are peers; each
    serves its own requests)."""

    def __init__(self, model: str, device, max_batch: int = 256, max_model_len: int = 2048,
                 seed: int = 0, num_blocks: Optional[int] = None, dtype=torch.bfloat16,
                 max_prefill_tokens: int = 16384, lookahead: Optional[bool] = None,
                 comm: Optional[str] = None, model_dir: Optional[str] = None):
        from .transport import init_distributed
        dev = torch.device(device)
        self.rank, self.world = init_distributed(device=dev if dev.type == "cuda" else None)
        cfg = get_config(model) if model_dir is None else _dir_config(model_dir, model)
        if not cfg.is_moe:
            raise ValueError(f"{model} has no experts")
        self.cfg = cfg
        from datetime import timedelta
        from .transport import resolve_comm
        self.ctrl_group = dist.new_group(backend="gloo", timeout=timedelta(days=365))
        # "auto" (default): the device mailboxes when every rank is a GPU process on this
        # host and they pass their self-test, else the torch all-to-all (resolve_comm)
        requested = comm or os.environ.get("DLI_EP_COMM", "auto")
        self.comm = resolve_comm(requested, dev, self.ctrl_group)
        self.fallback: Optional[str] = None
        self.moe = ExpertParallelMoE(cfg.num_experts, cfg.top_k_experts)
        er = self.moe.expert_range()
        if model_dir is not None:
            params = load_ep_params(model_dir, cfg, er, dev, dtype)
        else:
            shapes = W.stage_param_shapes(cfg, 0, cfg.num_layers, True, True)
            params = {}
            # generate full tensors per name (deterministic) and keep only the local experts
            for name, shape in shapes.items():
                t = W.random_init({name: shape}, dev, dtype, seed)[name]
                params[name] = W.slice_experts(name, t, er)
                del t
        lm = TransformerLM(cfg, params, device=dev, expert_range=er)
        lm.moe_fn = self.moe
        ipc = self.comm == "ipc"
        if ipc:
            from .transport import ipc_selftest
            self.moe.setup_ipc(dev, cfg.hidden_size, dtype,
                               max(max_prefill_tokens, max_batch), max_batch)
            if not ipc_selftest(self.moe.ep, self.ctrl_group):
                if requested == "ipc":
                    raise RuntimeError("IPC expert data plane failed its self-test")
                self.moe.close()
                self.comm, ipc = "torch", False
                self.fallback = "ipc self-test failed"
                _log.warning("expert-parallel rank %d: IPC mailboxes failed their self-test; "
                             "the all-to-all falls back to torch.distributed (%s)",
                             self.rank, dist.get_backend())
        from .transport import data_plane_name
        self.data_plane = data_plane_name(
            self.comm, dist.get_backend() == "nccl" or (ipc and dev.type == "cuda"))
        # with the mailbox data plane the decode forward is captured (graphs); the torch
        # data plane needs host-side split sizes per layer and runs eagerly
        graphs = ipc and dev.type == "cuda" and os.environ.get("DLI_NO_GRAPHS", "0") != "1"
        self.engine = LLMEngine(cfg, device=str(dev), dtype=dtype, max_batch=max_batch,
                                max_model_len=max_model_len, num_blocks=num_blocks,
                                use_graphs=graphs, lm=lm,
                                max_prefill_tokens=max_prefill_tokens, lookahead=lookahead,
                                mixed_steps=False)
        self.max_batch = max_batch
        self.device = dev
        self.steps = 0
        self.graph_steps = 0
        self.lockstep_syncs = 0
        # a rank whose peers are decoding admits prompts in chunks of at most max_batch
        # tokens, so the step stays within the peers' captured receive regions and they keep
        # replaying their decode graphs (a larger prefill sends every rank eager for that
        # step); DLI_EP_PREFILL_CAP=0 turns it off
        self.prefill_cap = os.environ.get("DLI_EP_PREFILL_CAP", "1") == "1"
        self._full_prefill = self.engine.scheduler.max_prefill_tokens
        self._peers_decoding = False
        self.capped_steps = 0
        # serving: a rank asks the group to stop (ExpertService.close); every rank learns it
        # from the lockstep exchange and leaves the loop once no rank has work
        self.stop_requested = False
        self.stopping = False
        # lockstep control plane: the shared-memory board when every rank is on this host
        # (the single-node deployment), else the gloo all_gather; host seconds spent in it
        self.board = self._open_board()
        self.control_plane = "shm" if self.board is not None else "gloo"
        self.lockstep_s = 0.0
        # liveness watchdog: a peer that dies mid-forward would leave this rank's
        # queue spinning in its mailbox waits for the whole wait budget; the board knows every
        # rank's pid, so a death aborts the mailboxes within ~0.2 s and the next step raises
        self.dead_peer: Optional[str] = None
        self._wd_stop = threading.Event()
        self._wd = None
        if self.board is not None:
            self._wd = threading.Thread(target=self._watch, args=(0.2,), daemon=True,
                                        name=f"dli-ep-watchdog-{self.rank}")
            self._wd.start()

    def _watch(self, period: float) -> None:
        while not self._wd_stop.wait(period):
            board = self.board
            d = board.dead() if board is not None else -1
            if d < 0 or d == self.rank:
                continue
            self.dead_peer = f"expert-parallel rank {d} exited"
            ep = self.moe.ep
            if ep is not None and hasattr(ep, "abort"):
                try:
                    ep.abort(5.0)
                except Exception:  # noqa: BLE001
                    pass
            board.close()               # a lockstep exchange blocked on it returns
            return

    def _open_board(self):
        """A ``LockstepBoard`` shared by every rank of the group, or None when the ranks span
        hosts (or the runtime library is unavailable)."""
        import socket
        hosts = [None] * self.world
        dist.all_gather_object(hosts, socket.gethostname(), group=self.ctrl_group)
        # DLI_EP_CTRL=gloo keeps the socket all_gather (A/B of the control plane, like
        # DLI_PP_CTRL for the pipeline)
        if (self.world == 1 or len(set(hosts)) != 1
                or os.environ.get("DLI_EP_CTRL", "auto") == "gloo"):
            return None
        try:
            from ..runtime import LockstepBoard
            name = [f"/dli_ep_board_{os.environ.get('MASTER_PORT', '0')}_{os.getpid()}"
                    if self.rank == 0 else None]
            board = LockstepBoard.create(name[0], self.world) if self.rank == 0 else None
            dist.broadcast_object_list(name, src=0, group=self.ctrl_group)
            if board is None:
                board = LockstepBoard.open(name[0])
            board.join(self.rank)
            dist.barrier(group=self.ctrl_group)
            if self.rank == 0:
                board.unlink()
            return board
        except (OSError, RuntimeError) as e:
            _log.warning("expert-parallel rank %d: shared-memory lockstep board unavailable "
                         "(%s); the lockstep exchange uses gloo", self.rank, e)
            return None

    def ring_bell(self) -> None:
        """Wake every rank sleeping in ``wait_bell`` (a request arrived, or a stop)."""
        if self.board is not None:
            self.board.ring()

    def bell(self) -> int:
        return self.board.bell() if self.board is not None else 0

    def wait_bell(self, seen: int, timeout_s: float) -> None:
        """Idle: sleep until some rank rings the doorbell (without the board: ``timeout_s``
        capped at a short poll period)."""
        if self.board is not None:
            self.board.wait_bell(seen, timeout_s)
        else:
            time.sleep(min(timeout_s, 0.002))

    def warmup(self):
        """Capture the decode graphs (every rank, same bucket order: the warm-up forwards
        inside each capture exchange with the peers)."""
        run = self.engine.runner
        if not run.use_graphs:
            return
        if os.environ.get("DLI_GEMM_AUTOTUNE", "1") == "1":
            # every bucket tuned before the first captured exchange (ranks sharing a GPU tune
            # one at a time: StageRunner.tune_lock), then all ranks start capturing together
            run.autotune(run.buckets)
            dist.barrier(group=self.ctrl_group)
        self.moe.static = True
        try:
            for b in run.buckets:
                self.moe.begin_step([b] * self.world)
                run.capture([b])
        finally:
            self.moe.static = False

    def _exchange(self, work: bool, tokens: int) -> List[List[int]]:
        """The per-step lockstep exchange: (has work, tokens of the next forward, stop) of
        every rank, host to host over the gloo control group. It never waits on a GPU: an
        RCCL all-gather read back with ``.tolist()`` would drain this rank's stream (the
        in-flight step included) before the next step could even be planned, defeating
        lookahead; the routing itself stays on the device (mailbox headers)."""
        t0 = time.perf_counter()
        words = [1 if work else 0, tokens, 1 if self.stop_requested else 0]
        if self.board is not None:
            rows = self.board.exchange(words).tolist()
        else:
            mine = torch.tensor(words, dtype=torch.int64)
            allv = [torch.empty_like(mine) for _ in range(self.world)]
            dist.all_gather(allv, mine, group=self.ctrl_group)
            rows = torch.stack(allv).tolist()
        self.lockstep_syncs += 1
        self.lockstep_s += time.perf_counter() - t0
        if any(r[2] for r in rows):
            self.stopping = True
        return [r[:2] for r in rows]

    def _idle_forward(self):
        """Join every MoE exchange of one forward with zero local rows."""
        D = self.cfg.hidden_size
        h = torch.zeros(0, D, dtype=self.engine.model.params["embed"].dtype, device=self.device)
        for i in range(self.cfg.num_layers):
            self.moe(h, self.engine.model.layers[i], i)

    def step(self):
        """One lockstep iteration: plan this rank's step, exchange (work, tokens) with every
        rank, then launch the forward (an empty one when this rank has none) and apply the
        tokens of the step that completes. Returns (outputs, any rank had work)."""
        eng = self.engine
        if self.dead_peer is not None:
            from .transport import PeerDied
            raise PeerDied(self.dead_peer)
        if self.moe.ep is not None:
            bits = self.moe.ep.error()
            if bits:
                from .transport import DataPlaneError
                raise DataPlaneError(bits)
        sch = eng.scheduler
        capped = self.prefill_cap and self._peers_decoding
        sch.max_prefill_tokens = min(self._full_prefill, self.max_batch) if capped \
            else self._full_prefill
        meta = eng.plan_step()
        work = meta is not None or eng.has_work()
        info = self._exchange(work, 0 if meta is None else meta.num_tokens)
        if not any(w for w, _ in info):
            return eng.finish_step(None), False
        toks = [t for _, t in info]
        if capped and meta is not None and meta.kind != DECODE:
            self.capped_steps += 1
        # peers with a graph-sized step (decode, or a capped prefill) keep their graphs only
        # if this rank's next step stays graph-sized too
        self._peers_decoding = any(0 < t <= self.max_batch
                                   for r, (w, t) in enumerate(info) if r != self.rank and w)
        self.moe.begin_step(toks)
        # a captured decode graph sizes its receive regions for decode batches: when any
        # rank's step is larger (a prefill), every rank runs this step eagerly
        run = eng.runner
        run.force_eager = max(toks) > self.max_batch
        replayed = run.replays
        try:
            if meta is None:
                self._idle_forward()
            self.steps += 1
            out = eng.finish_step(meta)
        except Exception as e:
            if self.dead_peer is not None:      # stale rows after the abort: name the cause
                from .transport import PeerDied
                raise PeerDied(self.dead_peer) from e
            raise
        self.graph_steps += run.replays - replayed
        return out, True

    def run_until_idle(self):
        outs = []
        while True:
            o, more = self.step()
            outs.extend(o)
            if not more:
                break
        return outs

    def generate(self, prompts, params=None):
        rids = [self.engine.add_request(p, params) for p in prompts]
        done = {o.request_id: o for o in self.run_until_idle()}
        return [done[r] for r in rids]

    def shard_record(self, model_name: str) -> dict:
        """This rank as a worker shard row (``loaded_shards`` of /health): shard id = rank,
        metadata = the experts it holds. Every rank serves whole requests (DP attention), so
        the master balances across the shard holders by load."""
        e0, e1 = self.moe.expert_range()
        return {"model_name": model_name, "shard_id": self.rank, "path": f"ep{self.rank}",
                "metadata": {"model_name": model_name, "shard_id": self.rank,
                             "num_shards": self.world, "kind": "expert",
                             "experts": [e0, e1], "num_experts": self.cfg.num_experts,
                             "start_layer": 0, "end_layer": self.cfg.num_layers - 1,
                             "total_layers": self.cfg.num_layers}}

    def close(self) -> None:
        self._wd_stop.set()
        if self._wd is not None:
            self._wd.join(1.0)
        self.moe.close()
        if self.board is not None:
            self.board.close()


def _dir_config(model_dir: str, name: str):
    """Config of an exported model directory (ours or a HF checkpoint)."""
    import json
    from pathlib import Path
    from ..models.configs import ModelConfig
    from ..models.hf import config_from_hf, is_hf_dir
    d = Path(model_dir)
    if is_hf_dir(d):
        return config_from_hf(json.loads((d / "config.json").read_text()), name)
    for c in [d / "config.json"] + sorted(d.glob("shard_*/config.json")):
        if c.exists():
            return ModelConfig.from_dict(json.loads(c.read_text()))
    raise FileNotFoundError(f"{model_dir}: no config.json")


def load_ep_params(model_dir: str, cfg, expert_range, device, dtype):
    """This rank's tensors from an exported model (``shard-model`` output: every
    ``shard_<i>/model.safetensors``, or one ``model.safetensors``; or a HF checkpoint): all
    attention / norm / embedding / head tensors, and of every expert tensor only the rows of
    experts [e0, e1) — a contiguous byte range of the file (``SafetensorsFile.load_rows``), so
    a rank never reads the other ranks' experts."""
    from pathlib import Path
    from ..models.hf import is_hf_dir, load_hf_dir
    from ..runtime import SafetensorsFile
    d = Path(model_dir)
    e0, e1 = expert_range
    if is_hf_dir(d):
        _, full = load_hf_dir(d, "cpu", dtype)
        return {k: W.slice_experts(k, v, expert_range).to(device) for k, v in full.items()}
    files = sorted(d.glob("shard_*/model.safetensors")) or [d / "model.safetensors"]
    out = {}
    for f in files:
        st = SafetensorsFile(str(f))
        try:
            names = st.keys()
            experts = [n for n in names if n.endswith(".w_gu") or n.endswith(".w_down")]
            rest = [n for n in names if n not in experts]
            out.update(st.load(rest, device=device))
            for n in experts:
                out[n] = st.load_rows(n, e0, e1, device=device)
        finally:
            st.close()
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    return {k: (v if v.dtype == dtype else v.to(dtype)) for k, v in out.items()}


def bench_expert_parallel(args, world, rank, make_prompts):
    local = int(os.environ.get("LOCAL_RANK", rank))
    if os.environ.get("DLI_SAME_DEVICE", "0") == "1":
        local = 0
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    eng = ExpertParallelEngine(args.model, dev, max_batch=args.batch,
                               max_model_len=args.max_model_len,
                               max_prefill_tokens=max(args.batch * args.prompt_len, 8192),
                               model_dir=getattr(args, "shard_dir", None))
    eng.warmup()
    from ..engine.sequence import SamplingParams
    sp = SamplingParams(max_length=args.max_length, temperature=0.8, top_k=50, top_p=0.95,
                        ignore_eos=True)

    def wave(seed):
        outs = eng.generate(make_prompts(args.batch, args.prompt_len, eng.cfg.vocab_size,
                                         seed * 100 + rank), sp)
        return sum(len(o.output_ids) for o in outs), [o.latency_s for o in outs]

    for w in range(args.warmup):
        wave(10_000 + w)
    dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    eng.lockstep_s, eng.lockstep_syncs = 0.0, 0
    t0 = time.perf_counter()
    toks, lats = 0, []
    for s in range(args.steps):
        n, l = wave(s)
        toks += n
        lats += l
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dist.barrier()
    cdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=cdev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    tt = torch.tensor([toks], dtype=torch.float64, device=cdev)
    dist.all_reduce(tt)
    lat_t = torch.tensor(lats, dtype=torch.float64, device=cdev)
    gathered = [torch.zeros_like(lat_t) for _ in range(world)]
    dist.all_gather(gathered, lat_t)
    from .transport import gather_rank_info
    infos = gather_rank_info(dev)
    dist.barrier()
    eng.moe.close()
    dist.destroy_process_group()
    if rank != 0:
        return None
    return {"tokens": int(tt.item()), "seconds": float(dt.item()),
            "latencies": torch.cat(gathered).tolist(), "global_batch": args.batch * world,
            "parallelism": f"dp{world}-ep{world}", "data_plane": eng.data_plane,
            "ranks_info": infos,
            "engine": {"control_plane": eng.control_plane,
                       "lockstep_ms_per_step": round(1e3 * eng.lockstep_s
                                                     / max(1, eng.lockstep_syncs), 4),
                       "steps": eng.lockstep_syncs}}
