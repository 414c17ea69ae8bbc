"""Point-to-point transport between pipeline ranks.

Replaces the reference's RPC + CPU-staging transport
(``torchgpipe/distributed/gpipe.py:86-96``: ``to('cpu')`` → ``rpc.remote`` →
``Queue``) with GPU-direct ``torch.distributed`` point-to-point operations:
on ROCm the ``nccl`` backend *is* RCCL, so an activation, gradient or skip
tensor travels HBM → xGMI link → HBM with no host copy.  On CPU (tests) the
same code runs over ``gloo``.

Messages.  Everything that rank ``a`` sends to rank ``b`` for one micro-batch
in one direction forms a *message*: a list of tensors in a canonical order
known to both sides.  A message with one tensor is sent as is; a message with
several tensors (AmoebaNet's ``(x, skip)`` boundaries, or an activation plus
skip tensors bound for the same rank) is packed into one flat byte buffer by
the HIP segment-copy kernel (one RCCL send instead of several) and unpacked on
the receiver as zero-copy views into the received buffer.

Metadata.  Receivers must allocate buffers before posting a receive.
Shapes are exchanged once per (step signature, micro-batch, link, direction)
over a CPU ``gloo`` control group — so no GPU→host synchronisation is ever
needed — and cached afterwards.

Failure detection.  The reference blocks forever on a rank that died or sent
out of order (``torchgpipe/distributed/context.py:37``, "TODO: error
handling").  Here every host-side wait is bounded: gloo waits (metadata,
control payloads, host-staged tensors) take ``timeout`` and raise
:class:`PipelineTimeout` naming the peer and message, and RCCL waits are
stream-ordered, so a missing peer is caught by the process group's watchdog
(``init_process_group(timeout=...)``), which aborts the rank instead of
hanging the job.

Multi-path transfers.  With a stripe plan (``parallel/stripes.py``, set per step by the
pipeline stage) a large message leaves as pieces over the direct link and over detours
through idle ranks, which forward them (:meth:`P2P.begin_relays`).
"""
import contextlib
from dataclasses import dataclass, field
import datetime
import threading
from typing import Any, Dict, FrozenSet, Hashable, List, Optional, Sequence, Tuple

import torch
from torch import Tensor
import torch.distributed as dist

from torchgpipe_amd.ops import misc
from torchgpipe_amd.parallel.stripes import RelayJob, Send, message_kind, pieces

__all__ = ['TensorMeta', 'P2P', 'Message', 'PipelineTimeout', 'StripePlan']

_DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64,
           torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool]
_DTYPE_CODE = {d: i for i, d in enumerate(_DTYPES)}
_HEADER_LEN = 512


@dataclass(frozen=True)
class TensorMeta:
    shape: Tuple[int, ...]
    dtype: torch.dtype
    requires_grad: bool

    @staticmethod
    def of(t: Tensor) -> 'TensorMeta':
        return TensorMeta(tuple(t.shape), t.dtype, bool(t.requires_grad))

    @property
    def nbytes(self) -> int:
        n = 1
        for d in self.shape:
            n *= d
        return n * torch.empty((), dtype=self.dtype).element_size()


def encode_metas(metas: Sequence[TensorMeta], atomic: bool = False) -> Tensor:
    words: List[int] = [len(metas), int(atomic)]
    for m in metas:
        words += [_DTYPE_CODE[m.dtype], int(m.requires_grad), len(m.shape), *m.shape]
    if len(words) > _HEADER_LEN:
        raise ValueError('message metadata too large')
    header = torch.zeros(_HEADER_LEN, dtype=torch.int64)
    header[:len(words)] = torch.tensor(words, dtype=torch.int64)
    return header


def decode_metas(header: Tensor) -> Tuple[List[TensorMeta], bool]:
    words = header.tolist()
    count, atomic, pos = words[0], bool(words[1]), 2
    metas: List[TensorMeta] = []
    for _ in range(count):
        dtype = _DTYPES[words[pos]]
        grad = bool(words[pos + 1])
        ndim = words[pos + 2]
        shape = tuple(words[pos + 3:pos + 3 + ndim])
        pos += 3 + ndim
        metas.append(TensorMeta(shape, dtype, grad))
    return metas, atomic


class PipelineTimeout(RuntimeError):
    """A point-to-point wait exceeded the pipeline's timeout (dead or mis-ordered peer)."""


def _wait(work: object, timeout: Optional[datetime.timedelta], what: str) -> None:
    """``work.wait()`` bounded by ``timeout`` (host-blocking gloo works only)."""
    try:
        if timeout is None:
            work.wait()  # type: ignore[attr-defined]
        else:
            work.wait(timeout)  # type: ignore[attr-defined]
    except RuntimeError as exc:
        msg = str(exc)
        if 'imeout' in msg or 'imed out' in msg:
            raise PipelineTimeout(f'{what}: no matching peer operation within {timeout} '
                                  f'(peer dead or messages out of order): {msg}') from exc
        if 'onnection closed' in msg or 'onnection reset' in msg:
            # gloo closes a pair when one side's wait times out: the peer gave up (its own
            # timeout on a mis-ordered exchange) or died
            raise PipelineTimeout(f'{what}: the peer closed the connection (it died, or '
                                  f'timed out waiting on this rank): {msg}') from exc
        raise


def _align16(n: int) -> int:
    return (n + 15) // 16 * 16


def _bytes_of(t: Tensor) -> Tensor:
    """Flat byte view of a contiguous tensor (its pieces travel as slices of it)."""
    return t.reshape(-1).view(torch.uint8)


class Message:
    """Handle of a posted receive: ``wait()`` returns the received tensors."""

    __slots__ = ('_works', '_tensors', '_buffer', '_metas', 'atomic', '_device', '_timeout',
                 '_what', '_dest')

    def __init__(self, works: List[object], tensors: Optional[List[Tensor]],
                 buffer: Optional[Tensor], metas: List[TensorMeta], atomic: bool,
                 device: Optional[torch.device] = None,
                 timeout: Optional[datetime.timedelta] = None, what: str = '',
                 dest: Optional[List[Tensor]] = None) -> None:
        self._works = works
        self._timeout = timeout
        self._what = what
        self._tensors = tensors
        self._buffer = buffer
        self._metas = metas
        self.atomic = atomic
        # Host-staged receive (gloo transport for device tensors): move the
        # received host buffers onto this device after the wait -- into ``dest``
        # (persistent device buffers, same layout as the host ones) when given.
        self._device = device
        self._dest = dest

    def wait(self) -> List[Tensor]:
        """Wait (stream-ordered on GPUs) and return detached leaf tensors.

        Each leaf carries the sender's ``requires_grad`` flag, so received
        activations become the roots of this rank's backward graph.
        """
        for w in self._works:
            _wait(w, self._timeout, self._what)
        self._works = []
        if self._device is not None:
            if self._dest is not None:
                host = self._tensors if self._tensors is not None else [self._buffer]
                for d, h in zip(self._dest, host):  # type: ignore[arg-type]
                    d.copy_(h, non_blocking=True)
                if self._tensors is not None:
                    self._tensors = list(self._dest)
                else:
                    self._buffer = self._dest[0]
            else:
                if self._tensors is not None:
                    self._tensors = [t.to(self._device, non_blocking=True)
                                     for t in self._tensors]
                if self._buffer is not None:
                    self._buffer = self._buffer.to(self._device, non_blocking=True)
            self._device = None
        if self._tensors is None:
            assert self._buffer is not None
            views: List[Tensor] = []
            pos = 0
            for m in self._metas:
                nbytes = m.nbytes
                views.append(self._buffer[pos:pos + nbytes].view(m.dtype).view(m.shape))
                pos = _align16(pos + nbytes)
            self._tensors = views
        out = []
        for t, m in zip(self._tensors, self._metas):
            leaf = t.detach()
            if m.requires_grad:
                leaf.requires_grad_(True)
            out.append(leaf)
        return out


@dataclass
class StripePlan:
    """One step signature's multi-path transfers as seen by one rank."""
    # (src, dst) -> relays (global ranks), for every striped route of the pipeline
    stripes: Dict[Tuple[int, int], List[int]]
    # (src, dst) -> bytes of each message on the route, in order (the recorded step)
    sizes: Dict[Tuple[int, int], List[int]]
    # the routes this rank relays
    jobs: List[RelayJob] = field(default_factory=list)
    min_bytes: int = 0  # smaller messages of a striped route go direct
    sub: int = 4


class _Relay:
    """A relay's state for one route: a staging ring, the sends still reading it, and the
    stream (RCCL) its chains run on."""

    def __init__(self, slots: int) -> None:
        self.bufs: List[Optional[Tensor]] = [None] * slots
        self.pending: List[Optional[object]] = [None] * slots
        self.next = 0
        self.stream: Optional[torch.cuda.Stream] = None


class P2P:
    """RCCL/gloo point-to-point with cached shape metadata.

    Args:
        device: the device tensors are received on.
        group: process group for tensor traffic (``nccl`` = RCCL on GPUs).
        ctrl_group: ``gloo`` group for metadata (may equal ``group`` on CPU).
        timeout: bound (seconds) of every host-blocking wait; ``None`` = the
            process group's own timeout.
    """

    def __init__(self, device: torch.device, group: Optional[dist.ProcessGroup] = None,
                 ctrl_group: Optional[dist.ProcessGroup] = None,
                 pack: bool = True,
                 link_groups: Optional[Dict[int, dist.ProcessGroup]] = None,
                 timeout: Optional[float] = None) -> None:
        self.device = device
        self.timeout = None if timeout is None else datetime.timedelta(seconds=timeout)
        self.group = group
        # One 2-rank communicator per peer ("link"): RCCL then runs every link on
        # its own stream, so a send waiting for a slow peer never holds back
        # traffic to another peer (an eagerly initialised default group would
        # serialise all unbatched point-to-point ops on one stream).
        self.link_groups = link_groups or {}
        self.ctrl_group = ctrl_group
        self.pack = pack
        # gloo cannot move device memory: when the tensor transport is gloo and
        # the stage runs on a GPU (single-GPU rehearsal of a multi-rank run),
        # stage every message through host memory.
        self.stage_host = (device.type == 'cuda' and dist.is_initialized()
                           and dist.get_backend(group) == 'gloo')
        # Tensor works block the host only on gloo (RCCL waits are stream-ordered).
        self._host_waits = not dist.is_initialized() or dist.get_backend(group) == 'gloo' \
            or device.type != 'cuda'
        self._meta: Dict[Hashable, Tuple[List[TensorMeta], bool]] = {}
        # persistent receive buffers (recv(..., persistent=True)), per message key
        self._bufs: Dict[Hashable, List[Tensor]] = {}
        self._pending_sends: List[object] = []
        self._pending_meta: List[object] = []
        # multi-path transfers: this step's plan, per-route message counters, relay links
        # (one 2-rank group per detour pair) and relay states
        self.me = dist.get_rank() if dist.is_initialized() else 0
        self.plan: Optional[StripePlan] = None
        self._route_pos: Dict[Tuple[int, int], int] = {}
        self.relay_links: Dict[FrozenSet[int], Any] = {}
        self._relays: Dict[Tuple[int, int], _Relay] = {}
        self._relay_threads: List[threading.Thread] = []
        self._relay_errors: List[BaseException] = []
        self._recording: Optional[List[Send]] = None

    # -- metadata ---------------------------------------------------------------------------

    def _send_meta(self, metas: Sequence[TensorMeta], atomic: bool, dst: int) -> None:
        # Non-blocking: a blocking gloo send could wait on a receiver that is
        # itself waiting for an upstream rank.
        self._pending_meta.append(dist.isend(encode_metas(metas, atomic), dst,
                                             group=self.ctrl_group))

    def _recv_meta(self, src: int, key: Hashable) -> Tuple[List[TensorMeta], bool]:
        header = torch.empty(_HEADER_LEN, dtype=torch.int64)
        _wait(dist.irecv(header, src, group=self.ctrl_group), self.timeout,
              f'metadata of message {key!r} from rank {src}')
        return decode_metas(header)

    def send_control(self, payload: Tensor, dst: int) -> None:
        """Non-blocking send of a small CPU int64 tensor on the control group."""
        self._pending_meta.append(dist.isend(payload, dst, group=self.ctrl_group))

    def recv_control(self, payload: Tensor, src: int) -> Tensor:
        _wait(dist.irecv(payload, src, group=self.ctrl_group), self.timeout,
              f'control message from rank {src}')
        return payload

    def known(self, key: Hashable) -> Optional[Tuple[List[TensorMeta], bool]]:
        return self._meta.get(key)

    def forget(self) -> None:
        self._meta.clear()
        self._bufs.clear()

    # -- tensors ----------------------------------------------------------------------------

    def send(self, tensors: Sequence[Tensor], dst: int, key: Hashable,
             atomic: bool = False, cache: bool = True) -> None:
        """Send ``tensors`` to ``dst``.  Asynchronous for the host (RCCL).

        ``cache=False`` is for one-shot keys (e.g. per-iteration targets): the
        metadata travels with this message and is not remembered.
        """
        if not tensors:
            return
        metas = [TensorMeta.of(t) for t in tensors]
        cached = self._meta.get(key)
        if cached is None:
            self._send_meta(metas, atomic, dst)
            if cache:
                self._meta[key] = (metas, atomic)
        elif cached != (metas, atomic):
            raise RuntimeError(
                f'message {key!r} changed shape/dtype under the same step signature '
                f'({cached} -> {metas}); the receiver would misinterpret it')
        self._prune()
        single = len(tensors) == 1
        if self._recording is not None:
            kind = message_kind(key) if single or self.pack else 'unpacked'
            nbytes = metas[0].nbytes if single else self._packed_nbytes(metas)
            self._recording.append(Send(dst, kind or 'other', nbytes))
        if single or not self.pack:
            for t in tensors:
                t = t.detach().contiguous()
                if self.stage_host:
                    t = t.cpu()
                if single and self._striped(self.me, dst, t.numel() * t.element_size(), key):
                    self._send_pieces(_bytes_of(t), dst)
                    return
                self._pending_sends.append(dist.isend(t, dst, group=self._link(dst)))
            return
        buf = torch.empty(self._packed_nbytes(metas), dtype=torch.uint8, device=tensors[0].device)
        misc.pack([t.detach() for t in tensors], buf)
        if self.stage_host:
            buf = buf.cpu()
        if self._striped(self.me, dst, buf.numel(), key):
            self._send_pieces(buf, dst)
            return
        self._pending_sends.append(dist.isend(buf, dst, group=self._link(dst)))

    def recv(self, src: int, key: Hashable, cache: bool = True,
             persistent: bool = False) -> Message:
        """Post a receive from ``src``; the returned handle's ``wait()`` yields tensors.

        ``persistent``: receive into buffers kept per ``key`` and reused by every later
        receive of that key, so the tensors of a message sit at the same addresses each
        step (captured cell graphs read them in place, ``parallel/segments.py``).  The
        caller orders a new receive after the last reader of the previous one (the
        pipeline posts receives from its main stream, which has joined every lane by then).
        """
        cached = self._meta.get(key)
        if cached is None:
            cached = self._recv_meta(src, key)
            if cache:
                self._meta[key] = cached
        metas, atomic = cached
        if not metas:
            return Message([], [], None, metas, atomic)
        where = torch.device('cpu') if self.stage_host else self.device
        late = self.device if self.stage_host else None
        timeout = self.timeout if self._host_waits else None
        what = f'message {key!r} from rank {src}'
        split = len(metas) == 1 or not self.pack
        keep = self._persistent(key, metas, split) if persistent else None
        if split:
            out = ([torch.empty(m.shape, dtype=m.dtype, device=where) for m in metas]
                   if keep is None or self.stage_host else list(keep))
            if len(out) == 1 and self._striped(src, self.me, metas[0].nbytes, key):
                works = self._recv_pieces(_bytes_of(out[0]), src)
            else:
                works = [dist.irecv(t, src, group=self._link(src)) for t in out]
            return Message(works, out, None, metas, atomic, late, timeout, what,
                           keep if self.stage_host else None)
        buf = (torch.empty(self._packed_nbytes(metas), dtype=torch.uint8, device=where)
               if keep is None or self.stage_host else keep[0])
        works = (self._recv_pieces(buf, src) if self._striped(src, self.me, buf.numel(), key)
                 else [dist.irecv(buf, src, group=self._link(src))])
        return Message(works, None, buf, metas, atomic, late, timeout, what,
                       keep if self.stage_host else None)

    # -- multi-path transfers ---------------------------------------------------------------

    def start_recording(self) -> None:
        """Record every message sent from now on (destination, kind, bytes)."""
        self._recording = []

    def stop_recording(self) -> List[Send]:
        sends, self._recording = self._recording or [], None
        return sends

    def use_plan(self, plan: Optional[StripePlan]) -> None:
        """The stripe plan of the step about to run (``None``: every message direct)."""
        self.plan = plan
        self._route_pos = {}

    def _striped(self, src: int, dst: int, nbytes: int, key: Hashable) -> bool:
        """Whether this message of route ``src -> dst`` travels in pieces (checks it is the
        message the plan expects next on the route)."""
        plan = self.plan
        if plan is None or (src, dst) not in plan.stripes or nbytes < plan.min_bytes:
            return False
        sizes = plan.sizes[(src, dst)]
        pos = self._route_pos.get((src, dst), 0)
        if pos >= len(sizes) or sizes[pos] != nbytes:
            want = sizes[pos] if pos < len(sizes) else 'no message'
            raise RuntimeError(
                f'striped route {src} -> {dst}: message #{pos} ({key!r}) has {nbytes} bytes '
                f'but the stripe plan (recorded in the first step of this signature) expects '
                f'{want}; the step sends differently from the step it was planned on')
        self._route_pos[(src, dst)] = pos + 1
        return True

    def _pieces(self, peer: int, nbytes: int, src: int, dst: int
                ) -> List[Tuple[int, int, int, Optional[Any]]]:
        assert self.plan is not None
        relays = self.plan.stripes[(src, dst)]
        out = []
        for off, n, path in pieces(nbytes, len(relays), self.plan.sub):
            if path == 0:
                out.append((off, n, peer, self._link(peer)))
            else:
                r = relays[path - 1]
                out.append((off, n, r, self.relay_links[frozenset((self.me, r))]))
        return out

    def _send_pieces(self, flat: Tensor, dst: int) -> None:
        for off, n, peer, group in self._pieces(dst, flat.numel(), self.me, dst):
            self._pending_sends.append(dist.isend(flat[off:off + n], peer, group=group))

    def _recv_pieces(self, flat: Tensor, src: int) -> List[object]:
        return [dist.irecv(flat[off:off + n], peer, group=group)
                for off, n, peer, group in self._pieces(src, flat.numel(), src, self.me)]

    def begin_relays(self) -> None:
        """Post this step's relay chains: for every route this rank relays, each piece of
        every forward message is received from the source and sent on to the destination,
        then each piece of the gradients the other way.  RCCL: stream-ordered on one stream
        per route (the host returns at once); gloo: one thread per route."""
        if self.plan is None:
            return
        self._join_relays()
        for index, job in enumerate(self.plan.jobs):
            ops = ([(job.src, job.dst, n) for n in job.forward]
                   + [(job.dst, job.src, n) for n in job.backward])
            state = self._relays.get((job.src, job.dst))
            if state is None:
                state = self._relays[(job.src, job.dst)] = _Relay(4)
            size = max((n for _, _, n in ops), default=0)
            if self._host_waits:
                where = torch.device('cpu')
            else:
                where = self.device
                if state.stream is None:  # (named: a fixed stream set per process)
                    from torchgpipe_amd.stream import named_stream
                    state.stream = named_stream(self.device, f'relay-route{index}')
            # (re)allocate the ring on the route's stream, after the sends still reading it
            with (torch.cuda.stream(state.stream) if state.stream is not None
                  else contextlib.nullcontext()):
                for k, b in enumerate(state.bufs):
                    if b is None or b.numel() < size:
                        if state.pending[k] is not None:
                            _wait(state.pending[k], self.timeout if self._host_waits else None,
                                  'relay send')
                            state.pending[k] = None
                        state.bufs[k] = torch.empty(size, dtype=torch.uint8, device=where)
            if self._host_waits:
                t = threading.Thread(target=self._relay_chain, args=(ops, state),
                                     name=f'relay {job.src}->{job.dst}', daemon=True)
                t.start()
                self._relay_threads.append(t)
            else:
                with torch.cuda.stream(state.stream):
                    self._relay_chain(ops, state)

    def _relay_chain(self, ops: List[Tuple[int, int, int]], state: _Relay) -> None:
        host = self._host_waits
        timeout = self.timeout if host else None
        try:
            for src, dst, n in ops:
                slot = state.next
                state.next = (slot + 1) % len(state.bufs)
                prev = state.pending[slot]
                if prev is not None:  # the slot's previous send has left (RCCL: stream wait)
                    _wait(prev, timeout, 'relay send')
                buf = state.bufs[slot][:n]  # type: ignore[index]
                _wait(dist.irecv(buf, src, group=self.relay_links[frozenset((self.me, src))]),
                      timeout, f'relayed piece from rank {src} to rank {dst}')
                state.pending[slot] = dist.isend(
                    buf, dst, group=self.relay_links[frozenset((self.me, dst))])
            if host:
                for k, w in enumerate(state.pending):
                    if w is not None:
                        _wait(w, timeout, 'relay send')
                        state.pending[k] = None
        except BaseException as exc:  # surfaced by end_relays on the main thread
            if not host:
                raise
            self._relay_errors.append(exc)

    def _join_relays(self) -> None:
        threads, self._relay_threads = self._relay_threads, []
        for t in threads:
            t.join()
        errors, self._relay_errors = self._relay_errors, []
        if errors:
            raise errors[0]

    def end_relays(self) -> None:
        """Join the gloo relay threads of the step (re-raising their errors) and check that
        every striped route sent as many messages as planned."""
        self._join_relays()
        plan = self.plan
        if plan is not None:
            for (src, dst), sizes in plan.sizes.items():
                if src == self.me and (src, dst) in plan.stripes and \
                        self._route_pos.get((src, dst), 0) != len(sizes):
                    raise RuntimeError(
                        f'striped route {src} -> {dst} sent {self._route_pos.get((src, dst), 0)} '
                        f'messages this step, the stripe plan {len(sizes)}')
            self._route_pos = {}

    def _persistent(self, key: Hashable, metas: Sequence[TensorMeta],
                    split: bool) -> List[Tensor]:
        """The device buffers of ``key``'s persistent receives (allocated on first use)."""
        bufs = self._bufs.get(key)
        if bufs is None:
            if split:
                bufs = [torch.empty(m.shape, dtype=m.dtype, device=self.device) for m in metas]
            else:
                bufs = [torch.empty(self._packed_nbytes(metas), dtype=torch.uint8,
                                    device=self.device)]
            self._bufs[key] = bufs
        return bufs

    def _link(self, peer: int) -> Optional[dist.ProcessGroup]:
        return self.link_groups.get(peer, self.group)

    @staticmethod
    def _packed_nbytes(metas: Sequence[TensorMeta]) -> int:
        pos = 0
        for m in metas:
            pos = _align16(pos + m.nbytes)
        return max(pos, 16)

    def _prune(self) -> None:
        """Drop handles of sends that already completed (releases their buffers)."""
        if len(self._pending_sends) > 8:
            self._pending_sends = [w for w in self._pending_sends
                                   if not w.is_completed()]  # type: ignore[attr-defined]

    def flush(self) -> None:
        """Order the current stream after every send issued so far, release them."""
        timeout = self.timeout if self._host_waits else None
        for w in self._pending_sends:
            _wait(w, timeout, 'pending send')
        self._pending_sends = []
        for w in self._pending_meta:
            _wait(w, self.timeout, 'pending metadata send')
        self._pending_meta = []
