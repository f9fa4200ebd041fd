"""Siddhi-runtime-shaped Python wrapper over libcep (C ABI).

`SiddhiAppRuntime` mirrors the Siddhi calls flink-siddhi makes
(SURVEY.md §8b): getInputHandler / InputHandler.send, addCallback, snapshot,
shutdown — but batched and columnar: rows go in as numpy arrays (host) or
torch CUDA tensors (device-resident), matches come out through callbacks at
flush(), in Siddhi's emission order.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from . import _lib as L


def validate(plan: str) -> None:
    """SiddhiManager.validateSiddhiApp (AbstractSiddhiOperator.java:292-299)."""
    err = C.create_string_buffer(1024)
    rc = L.lib().cep_validate(plan.encode(), err, len(err))
    L.raise_for(rc, err.value.decode())


def plan_schema(plan: str, stream_id: str):
    """SiddhiTypeFactory.getStreamDefinition (utils/SiddhiTypeFactory.java:64-84):
    [(name, type_name)] of any input or output stream of `plan`."""
    err = C.create_string_buffer(1024)
    attrs = (L.cep_attr * 64)()
    n = C.c_int(0)
    rc = L.lib().cep_plan_schema(plan.encode(), stream_id.encode(), attrs, 64,
                                 C.byref(n), err, len(err))
    L.raise_for(rc, err.value.decode())
    return [(attrs[i].name.decode(), L.TYPE_NAMES[attrs[i].type])
            for i in range(n.value)]


@dataclass
class OutputRows:
    stream_id: str
    ts: np.ndarray
    seq: np.ndarray
    cols: List[np.ndarray]

    def __len__(self):
        return len(self.ts)

    def rows(self):
        return [tuple(c[i].item() for c in self.cols) for i in range(len(self.ts))]


class SiddhiAppRuntime:
    """createSiddhiAppRuntime(plan) + start() (AbstractSiddhiOperator.java:120-142)."""

    def __init__(self, plan: str, **options):
        self._lib = L.lib()
        self.options = L.default_options(**options)
        err = C.create_string_buffer(2048)
        h = self._lib.cep_create(plan.encode(), C.byref(self.options), err, len(err))
        if not h:
            msg = err.value.decode()
            # map the creation failure onto the reference's exception family
            code = L.CEP_E_PARSE
            vrc = self._lib.cep_validate(plan.encode(), None, 0)
            if vrc != L.CEP_OK:
                code = vrc
            elif "device" in msg.lower() or "gfx950" in msg or "HIP" in msg:
                code = L.CEP_E_DEVICE
            elif "capacity" in msg.lower() or "pending_slots" in msg:
                code = L.CEP_E_CAPACITY
            elif "not yet" in msg or "not supported" in msg:
                code = L.CEP_E_UNSUPPORTED
            L.raise_for(code, msg)
        self._h = C.c_void_p(h)
        self._owned = True
        self._callbacks: Dict[str, object] = {}
        self._collected: Dict[str, List[OutputRows]] = {}

    @classmethod
    def _borrow(cls, handle: int, options) -> "SiddhiAppRuntime":
        """A view of a runtime owned elsewhere (a plan of an operator.SiddhiOperator)."""
        r = cls.__new__(cls)
        r._lib = L.lib()
        r.options = options
        r._h = C.c_void_p(handle)
        r._owned = False
        r._callbacks = {}
        r._collected = {}
        return r

    # -- lifecycle -----------------------------------------------------------
    def shutdown(self):
        if self._h and self._owned:
            self._lib.cep_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.shutdown()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != L.CEP_OK:
            L.raise_for(rc, self._lib.cep_last_error(self._h).decode())

    # -- schema ----------------------------------------------------------------
    def stream_definition(self, stream_id: str):
        attrs = (L.cep_attr * 64)()
        n = C.c_int(0)
        self._check(self._lib.cep_stream_schema(self._h, stream_id.encode(),
                                                attrs, 64, C.byref(n)))
        return [(attrs[i].name.decode(), attrs[i].type) for i in range(n.value)]

    def input_handle(self, stream_id: str) -> int:
        h = self._lib.cep_input(self._h, stream_id.encode())
        if h < 0:
            self._check(-h)
        return h

    def intern(self, s: str) -> int:
        return self._lib.cep_dict_intern(self._h, s.encode())

    def lookup(self, i: int) -> Optional[str]:
        r = self._lib.cep_dict_lookup(self._h, int(i))
        return None if r is None else r.decode()

    # -- callbacks -------------------------------------------------------------
    def add_callback(self, out_id: str,
                     fn: Optional[Callable[[OutputRows], None]] = None, copy: bool = True):
        """addCallback(outId, StreamCallback) (AbstractSiddhiOperator.java:165-166).
        Without `fn`, rows are collected and returned by `collect(out_id)`.
        copy=False hands `fn` views of the engine's (pinned) delivery buffers,
        valid only during the call."""
        types = [t for _, t in self.stream_definition(out_id)]
        self._collected.setdefault(out_id, [])

        def cb(user, rows_p):
            r = rows_p.contents
            n = r.n
            cp = (lambda x: x.copy()) if copy or fn is None else (lambda x: x)
            ts = cp(np.ctypeslib.as_array(r.ts, shape=(n,))) if n else np.zeros(0, np.int64)
            # seq is NULL under options.omit_seq (not delivered)
            seq = cp(np.ctypeslib.as_array(r.seq, shape=(n,))) if n and r.seq else np.zeros(0, np.int64)
            cols = []
            for c, t in enumerate(types):
                dt = np.dtype(L.NUMPY_DTYPES[t])
                if n:
                    buf = (C.c_char * (n * dt.itemsize)).from_address(r.cols[c])
                    cols.append(cp(np.frombuffer(buf, dtype=dt)))
                else:
                    cols.append(np.zeros(0, dt))
            out = OutputRows(out_id, ts, seq, cols)
            if fn is not None:
                fn(out)
            else:
                self._collected[out_id].append(out)

        cfn = L.EMIT_FN(cb)
        self._callbacks[out_id] = cfn
        self._check(self._lib.cep_set_callback(self._h, out_id.encode(), cfn, None))

    def collect(self, out_id: str) -> OutputRows:
        parts = self._collected.get(out_id, [])
        self._collected[out_id] = []
        types = [t for _, t in self.stream_definition(out_id)]
        if not parts:
            return OutputRows(out_id, np.zeros(0, np.int64), np.zeros(0, np.int64),
                              [np.zeros(0, L.NUMPY_DTYPES[t]) for t in types])
        return OutputRows(out_id, np.concatenate([p.ts for p in parts]),
                          np.concatenate([p.seq for p in parts]),
                          [np.concatenate([p.cols[c] for p in parts])
                           for c in range(len(types))])

    # -- input -----------------------------------------------------------------
    def send(self, stream_id: str, ts, cols: Sequence, streams=None):
        """A batch of InputHandler.send(ts, row) (AbstractSiddhiOperator.java:130).

        `cols` follow the stream definition's attribute order.  numpy arrays
        are host batches (staged over PCIe); torch CUDA tensors are
        device-resident.  `streams` (uint8 per row: input handles) mixes
        several identically-defined streams in one batch.
        """
        self._send(self._lib.cep_send_batch, stream_id, ts, cols, streams)

    def process_elements(self, stream_id: str, ts, cols: Sequence, streams=None):
        """Event-time input in any timestamp order: the rows are buffered on
        the device until a watermark releases them, as the operator's
        processElement offers records to its PriorityQueue
        (AbstractSiddhiOperator.java:222-231).  Same arguments as send()."""
        self._send(self._lib.cep_buffer_batch, stream_id, ts, cols, streams)

    def process_watermark(self, mark: int):
        """processWatermark (AbstractSiddhiOperator.java:238-247): buffered rows
        with ts <= mark reach the engine in (ts, arrival) order; later rows
        stay buffered.  A row older than one already released (a late event)
        is dropped and counted in stats().late_events; with the runtime
        option late_policy=1 the call then raises (after the release)."""
        self._check(self._lib.cep_watermark(self._h, int(mark)))

    def buffered(self) -> int:
        """Rows waiting for a watermark (the PriorityQueue's size)."""
        return int(self._lib.cep_buffered(self._h))

    def _send(self, fn, stream_id: str, ts, cols: Sequence, streams=None):
        h = self.input_handle(stream_id)
        defs = self.stream_definition(stream_id)
        on_device = _is_device(ts)
        keep = []
        ptrs = (C.c_void_p * max(1, len(cols)))()
        for i, c in enumerate(cols):
            want = np.dtype(L.NUMPY_DTYPES[defs[i][1]]) if i < len(defs) else None
            p, k = _ptr(c, want, on_device)
            ptrs[i] = p
            keep.append(k)
        tsp, k = _ptr(ts, np.dtype("int64"), on_device)
        keep.append(k)
        sp = None
        if streams is not None:
            sp, k = _ptr(streams, np.dtype("uint8"), on_device)
            keep.append(k)
        b = L.cep_batch(n=_len(ts), ts=tsp, stream=sp, input=h, ncols=len(cols),
                        cols=ptrs, on_device=1 if on_device else 0)
        if on_device:
            self._wait_producer(ts)
        self._check(fn(self._h, C.byref(b)))
        if on_device:
            self._signal_consumer(ts)

    def _wait_producer(self, t):
        """Order the engine's stream after torch's current stream (device
        inputs may still be in flight there: generators, copies, RCCL)."""
        import torch
        s = torch.cuda.current_stream(t.device).cuda_stream
        self._check(self._lib.cep_stream_wait(self._h, C.c_void_p(s)))

    def _signal_consumer(self, t):
        """Order torch's current stream after the engine's queued work: the
        caching allocator may hand a freed input tensor's memory to a later
        kernel on that stream, which must not run while the engine still reads
        it (cep.h, Ownership)."""
        import torch
        s = torch.cuda.current_stream(t.device).cuda_stream
        self._check(self._lib.cep_stream_signal(self._h, C.c_void_p(s)))

    def flush(self):
        self._check(self._lib.cep_flush(self._h))

    # -- multi-GPU key shuffle (router/HashPartitioner.java:24-26) ---------------
    def record_words(self) -> int:
        w = self._lib.cep_record_words(self._h)
        if w < 0:
            self._check(-w)
        return w

    def route(self, stream_id: str, ts, cols: Sequence, world: int, seq0: int,
              streams=None, out=None, wait: bool = True):
        """Sender side of the key shuffle: evaluates the pattern's state
        filters on a device batch (push-down) and returns (records, counts):
        a uint64 device tensor [n, record_words] grouped by owner shard
        (key % world) in arrival order, and the per-owner record counts.
        The routing is complete on return (the counts are read back).
        wait=False: the inputs are known to be ready (produced before an
        earlier sync), so routing does not queue behind torch's stream."""
        import torch
        h = self.input_handle(stream_id)
        defs = self.stream_definition(stream_id)
        if not _is_device(ts):
            raise ValueError("route() takes device-resident columns")
        keep = []
        ptrs = (C.c_void_p * max(1, len(cols)))()
        for i, c in enumerate(cols):
            p, k = _ptr(c, np.dtype(L.NUMPY_DTYPES[defs[i][1]]), True)
            ptrs[i] = p
            keep.append(k)
        sp = None
        if streams is not None:
            sp, k = _ptr(streams, np.dtype("uint8"), True)
            keep.append(k)
        n = _len(ts)
        w = self.record_words()
        if out is None or out.shape[0] < n:
            out = torch.empty((max(n, 1), w), dtype=torch.int64, device=ts.device)
        b = L.cep_batch(n=n, ts=C.c_void_p(ts.data_ptr()), stream=sp, input=h, ncols=len(cols),
                        cols=ptrs, on_device=1)
        counts = (C.c_int64 * world)()
        if wait:
            self._wait_producer(ts)
        self._check(self._lib.cep_route_batch(self._h, C.byref(b), world, seq0,
                                              C.c_void_p(out.data_ptr()), out.shape[0], counts))
        return out, [int(c) for c in counts]

    def route_padded(self, stream_id: str, ts, cols: Sequence, world: int, seq0: int, seg_cap: int,
                     streams=None, out=None, wait: bool = True, rows: bool = False, spill=None):
        """Padded sender side (cep_route_batch_padded; rows=True:
        cep_route_rows_padded): a uint64 device tensor [world * (1 + seg_cap),
        words] of fixed owner segments with the counts in-band (segment
        headers).  Nothing is read back: the route is only queued, so the step
        needs no host round trip.

        spill = (buffer [cap, words], counts [world] int64), device tensors:
        an owner's records past seg_cap go to the buffer instead of being
        dropped (cep_route_*_padded_spill; flink_siddhi.shuffle.PaddedShuffle
        ships them)."""
        import torch
        h = self.input_handle(stream_id)
        defs = self.stream_definition(stream_id)
        if not _is_device(ts):
            raise ValueError("route_padded() takes device-resident columns")
        keep = []
        ptrs = (C.c_void_p * max(1, len(cols)))()
        for i, c in enumerate(cols):
            p, k = _ptr(c, np.dtype(L.NUMPY_DTYPES[defs[i][1]]), True)
            ptrs[i] = p
            keep.append(k)
        sp = None
        if streams is not None:
            sp, k = _ptr(streams, np.dtype("uint8"), True)
            keep.append(k)
        nrows = world * (1 + int(seg_cap))
        w = self.row_words() if rows else self.record_words()
        if out is None or out.shape[0] < nrows or out.shape[1] != w:
            out = torch.empty((nrows, w), dtype=torch.int64, device=ts.device)
        b = L.cep_batch(n=_len(ts), ts=C.c_void_p(ts.data_ptr()), stream=sp, input=h, ncols=len(cols),
                        cols=ptrs, on_device=1)
        if wait:
            self._wait_producer(ts)
        if spill is None:
            fn = self._lib.cep_route_rows_padded if rows else self._lib.cep_route_batch_padded
            self._check(fn(self._h, C.byref(b), world, seq0, C.c_void_p(out.data_ptr()), out.shape[0],
                           int(seg_cap)))
        else:
            sbuf, scnt = spill
            if sbuf.shape[1] != w or scnt.numel() < world or scnt.dtype != torch.int64:
                raise ValueError("spill: buffer [cap, %d] and int64 counts [world]" % w)
            fn = self._lib.cep_route_rows_padded_spill if rows else self._lib.cep_route_batch_padded_spill
            self._check(fn(self._h, C.byref(b), world, seq0, C.c_void_p(out.data_ptr()), out.shape[0],
                           int(seg_cap), C.c_void_p(sbuf.data_ptr()), sbuf.shape[0],
                           C.c_void_p(scnt.data_ptr())))
        # torch's stream (the all-to-all) must not read the segments before the
        # route stream wrote them; the walk queued on the engine stream is not
        # waited for
        s = torch.cuda.current_stream(ts.device).cuda_stream
        self._check(self._lib.cep_route_signal(self._h, C.c_void_p(s)))
        return out[:nrows]

    def send_padded(self, segs, world: int, seg_cap: int, events_represented: int = 0,
                    signal: bool = True, rows: bool = False):
        """Owner side of the padded shuffle: the world received segments in
        source-rank order (rows=True: whole rows of the row shuffle).  An
        overflowed segment fails the next flush."""
        if getattr(segs, "is_cuda", False):
            self._wait_producer(segs)
        fn = self._lib.cep_send_rows_padded if rows else self._lib.cep_send_records_padded
        self._check(fn(self._h, C.c_void_p(segs.data_ptr()), world, int(seg_cap), events_represented))
        if signal and getattr(segs, "is_cuda", False):
            self._signal_consumer(segs)

    def partition_channels(self, stream_id: str, ts, cols: Sequence, key_field: Optional[str],
                           nchan: int, seq0: int = 0, keys: bool = False):
        """Dynamic-path routing of a device batch (AddRouteOperator.java:83-92 ->
        DynamicPartitioner.java:43-60 -> HashPartitioner.java:24-26): the
        channel of each row, |Java hashCode(key_field)| % nchan, as an int32
        device tensor (and the int64 partition keys with keys=True).  No
        key_field: key -1 and a pseudo-random channel."""
        import torch
        h = self.input_handle(stream_id)
        defs = self.stream_definition(stream_id)
        if not _is_device(ts):
            raise ValueError("partition_channels() takes device-resident columns")
        keep = []
        ptrs = (C.c_void_p * max(1, len(cols)))()
        for i, c in enumerate(cols):
            p, k = _ptr(c, np.dtype(L.NUMPY_DTYPES[defs[i][1]]), True)
            ptrs[i] = p
            keep.append(k)
        n = _len(ts)
        chan = torch.empty(max(n, 1), dtype=torch.int32, device=ts.device)
        kt = torch.empty(max(n, 1), dtype=torch.int64, device=ts.device) if keys else None
        b = L.cep_batch(n=n, ts=C.c_void_p(ts.data_ptr()), stream=None, input=h, ncols=len(cols),
                        cols=ptrs, on_device=1)
        self._wait_producer(ts)
        self._check(self._lib.cep_partition_channels(
            self._h, C.byref(b), key_field.encode() if key_field else None, int(nchan), int(seq0),
            C.c_void_p(chan.data_ptr()), C.c_void_p(kt.data_ptr()) if keys else None))
        self._signal_consumer(ts)
        return (chan[:n], kt[:n]) if keys else chan[:n]

    def row_words(self) -> int:
        w = self._lib.cep_row_words(self._h)
        if w < 0:
            self._check(-w)
        return w

    def route_rows(self, stream_id: str, ts, cols: Sequence, world: int, seq0: int,
                   streams=None, out=None, wait: bool = True):
        """Sender side of the row shuffle (multi-query apps, no push-down):
        (rows, counts) — an int64 device tensor [n, row_words] grouped by
        owner in arrival order, and the per-owner row counts."""
        import torch
        h = self.input_handle(stream_id)
        defs = self.stream_definition(stream_id)
        if not _is_device(ts):
            raise ValueError("route_rows() takes device-resident columns")
        keep = []
        ptrs = (C.c_void_p * max(1, len(cols)))()
        for i, c in enumerate(cols):
            p, k = _ptr(c, np.dtype(L.NUMPY_DTYPES[defs[i][1]]), True)
            ptrs[i] = p
            keep.append(k)
        sp = None
        if streams is not None:
            sp, k = _ptr(streams, np.dtype("uint8"), True)
            keep.append(k)
        n = _len(ts)
        w = self.row_words()
        if out is None or out.shape[0] < n:
            out = torch.empty((max(n, 1), w), dtype=torch.int64, device=ts.device)
        b = L.cep_batch(n=n, ts=C.c_void_p(ts.data_ptr()), stream=sp, input=h, ncols=len(cols),
                        cols=ptrs, on_device=1)
        counts = (C.c_int64 * world)()
        if wait:
            self._wait_producer(ts)
        self._check(self._lib.cep_route_rows(self._h, C.byref(b), world, seq0,
                                             C.c_void_p(out.data_ptr()), out.shape[0], counts))
        return out, [int(c) for c in counts]

    def send_rows(self, rows, n: int, events_represented: int = 0, signal: bool = True):
        """Owner side of the row shuffle: received rows in source-rank order."""
        p = C.c_void_p(rows.data_ptr()) if n else None
        if n and getattr(rows, "is_cuda", False):
            self._wait_producer(rows)
        self._check(self._lib.cep_send_rows(self._h, p, n, events_represented))
        if n and signal and getattr(rows, "is_cuda", False):
            self._signal_consumer(rows)

    def send_records(self, recs, n: int, events_represented: int = 0, signal: bool = True):
        """Owner side: feed received shuffle records (source-rank order).
        signal=False leaves torch's stream free to run ahead of the walk (the
        caller keeps `recs` alive and unchanged, e.g. double-buffered, and
        orders its reuse with signal())."""
        p = C.c_void_p(recs.data_ptr()) if n else None
        if n and getattr(recs, "is_cuda", False):
            self._wait_producer(recs)
        self._check(self._lib.cep_send_records(self._h, p, n, events_represented))
        if n and signal and getattr(recs, "is_cuda", False):
            self._signal_consumer(recs)

    def signal(self, stream):
        """Make a torch stream wait for the engine's work queued so far."""
        self._check(self._lib.cep_stream_signal(self._h, C.c_void_p(stream.cuda_stream)))

    def output_device(self, out_id: str):
        r = L.cep_rows()
        self._check(self._lib.cep_output_device(self._h, out_id.encode(), C.byref(r)))
        return r

    def output_tensors(self, out_id: str, copy: bool = True):
        """Device-resident consumer: the unflushed rows of out_id as torch
        CUDA tensors (ts, seq, [cols]) in device emission order (per-key
        order with ordered_output=0).  copy=False aliases engine memory that
        the next send / flush / reset_output invalidates."""
        import torch
        r = self.output_device(out_id)
        n = int(r.n)
        types = [t for _, t in self.stream_definition(out_id)]
        dev = torch.device("cuda", int(self.options.device))

        def wrap(ptr, dtype: str):
            t = torch.as_tensor(_DevArray(ptr, n, dtype), device=dev)
            return t.clone() if copy else t

        ts = wrap(C.cast(r.ts, C.c_void_p).value, "<i8")
        # None under omit_seq with unordered output (the kernels do not write them)
        seq_ptr = C.cast(r.seq, C.c_void_p).value
        seq = wrap(seq_ptr, "<i8") if seq_ptr else None
        cols = [wrap(r.cols[c], np.dtype(L.NUMPY_DTYPES[t]).str) for c, t in enumerate(types)]
        return ts, seq, cols

    def reset_output(self):
        self._check(self._lib.cep_reset_output(self._h))

    def set_enabled(self, enabled: bool):
        self._check(self._lib.cep_set_enabled(self._h, 1 if enabled else 0))

    # -- state -------------------------------------------------------------------
    def snapshot(self) -> bytes:
        buf = C.POINTER(C.c_uint8)()
        n = C.c_size_t(0)
        self._check(self._lib.cep_snapshot(self._h, C.byref(buf), C.byref(n)))
        try:
            return C.string_at(buf, n.value)
        finally:
            self._lib.cep_free(buf)

    def restore(self, data: bytes):
        b = C.create_string_buffer(data, len(data))
        self._check(self._lib.cep_restore(self._h, b, len(data)))

    def stats(self) -> L.cep_stats_t:
        s = L.cep_stats_t()
        self._check(self._lib.cep_stats(self._h, C.byref(s)))
        return s


class _DevArray:
    """A raw device buffer exposed through __cuda_array_interface__ (torch on
    ROCm reads the same protocol) so torch can view engine output memory."""

    def __init__(self, ptr, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr,
                                         "data": (int(ptr or 0), False), "version": 3,
                                         "strides": None}


def _is_device(x) -> bool:
    return hasattr(x, "is_cuda") and bool(x.is_cuda)


def _len(x) -> int:
    return int(x.shape[0]) if hasattr(x, "shape") else len(x)


def _ptr(x, want_dtype, on_device):
    if on_device:
        if not _is_device(x):
            raise ValueError("mixing host and device columns in one batch")
        return C.c_void_p(x.data_ptr()), x
    a = np.ascontiguousarray(x, dtype=want_dtype) if want_dtype is not None \
        else np.ascontiguousarray(x)
    return C.c_void_p(a.ctypes.data), a
