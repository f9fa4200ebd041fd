"""Dynamic execution plans: control events over one operator (libcep `cep_operator_*`).

Python mirror of flink-siddhi's dynamic path:

  * `MetadataControlEvent` / `OperationControlEvent` — control/MetadataControlEvent.java,
    control/OperationControlEvent.java (same builder, same actions),
  * `SiddhiOperator.on_event_received` — AbstractSiddhiOperator.onEventReceived
    (operator/AbstractSiddhiOperator.java:400-467): deleted plans first, then
    added, then updated; ENABLE_QUERY / DISABLE_QUERY pause and resume a plan,
  * `SiddhiOperator.process` — AddRouteOperator.processElement
    (router/AddRouteOperator.java:54-98): a batch of stream S reaches every
    enabled plan whose queries read S,
  * `SiddhiOperator.route` — the partition key (AddRouteOperator.java:83-92)
    and channel (router/DynamicPartitioner.java:43-60, HashPartitioner.java:24-26)
    of each row, computed on the GPU.

Plans are written without stream definitions and enriched with the data
streams' schemas, as SiddhiExecutionPlanner.getEnrichedExecutionPlan does
(utils/SiddhiExecutionPlanner.java:56-65).  Each plan is its own device
runtime, so changing one plan never touches another's state.
"""
from __future__ import annotations

import ctypes as C
import enum
import uuid
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .runtime import OutputRows, SiddhiAppRuntime, _is_device, _len, _ptr


class ControlEvent:
    """control/ControlEvent.java: marker base of the control stream."""

    def name(self) -> str:
        return type(self).__name__


class MetadataControlEvent(ControlEvent):
    """Plans added / updated / deleted (control/MetadataControlEvent.java)."""

    def __init__(self):
        self.added: Dict[str, str] = {}
        self.updated: Dict[str, str] = {}
        self.deleted: List[str] = []

    @staticmethod
    def next_execution_plan_id() -> str:
        return str(uuid.uuid4())

    @staticmethod
    def builder() -> "MetadataControlEvent.Builder":
        return MetadataControlEvent.Builder()

    class Builder:
        def __init__(self):
            self._ev = MetadataControlEvent()

        def add_execution_plan(self, plan_or_id: str, plan: Optional[str] = None):
            if plan is None:
                self._ev.added[MetadataControlEvent.next_execution_plan_id()] = plan_or_id
            else:
                self._ev.added[plan_or_id] = plan
            return self

        def remove_execution_plan(self, plan_id: str):
            self._ev.deleted.append(plan_id)
            return self

        def update_execution_plan(self, plan_id: str, plan: str):
            self._ev.updated[plan_id] = plan
            return self

        def build(self) -> "MetadataControlEvent":
            return self._ev


class OperationControlEvent(ControlEvent):
    """Pause / resume one plan (control/OperationControlEvent.java)."""

    class Action(enum.Enum):
        ENABLE_QUERY = 0
        DISABLE_QUERY = 1

    def __init__(self, action: "OperationControlEvent.Action", query_id: str):
        self.action = action
        self.query_id = query_id

    @staticmethod
    def enable_query(query_id: str) -> "OperationControlEvent":
        return OperationControlEvent(OperationControlEvent.Action.ENABLE_QUERY, query_id)

    @staticmethod
    def disable_query(query_id: str) -> "OperationControlEvent":
        return OperationControlEvent(OperationControlEvent.Action.DISABLE_QUERY, query_id)


def stream_definition_expression(stream_id: str, attrs: Sequence[Tuple[str, str]]) -> str:
    """SiddhiStreamSchema.getStreamDefinitionExpression (schema/SiddhiStreamSchema.java:63-71)."""
    return "define stream %s (%s);" % (stream_id, ", ".join("%s %s" % a for a in attrs))


def plan_input_streams(plan: str) -> List[str]:
    """Input streams the plan's queries read (the router's
    inputStreamToExecutionPlans, router/AddRouteOperator.java:159-175)."""
    buf = C.create_string_buffer(4096)
    rc = L.lib().cep_plan_input_streams(plan.encode(), buf, len(buf))
    L.raise_for(rc, buf.value.decode())
    v = buf.value.decode()
    return v.split("\n") if v else []


def plan_partition_keys(plan: str, stream_id: str) -> List[str]:
    """The group-by attributes that partition `stream_id` for `plan`
    (SiddhiExecutionPlanner.getStreamPartitions, utils/SiddhiExecutionPlanner.java:76-140)."""
    buf = C.create_string_buffer(4096)
    rc = L.lib().cep_plan_partition_keys(plan.encode(), stream_id.encode(), buf, len(buf))
    L.raise_for(rc, buf.value.decode())
    v = buf.value.decode()
    return v.split("\n") if v else []


class SiddhiOperator:
    """One operator hosting any number of execution plans (AbstractSiddhiOperator
    with its QueryRuntimeHandler map, :114-176), driven by control events.

    `data_stream_schemas`: stream id -> [(field, type)] of every data stream
    (SiddhiOperatorContext's SiddhiStreamSchema map), e.g.
    {"inputStream1": [("id", "int"), ("name", "string"), ("price", "double"),
    ("timestamp", "long")]}.
    """

    def __init__(self, data_stream_schemas: Dict[str, Sequence[Tuple[str, str]]], **options):
        self._lib = L.lib()
        self.schemas = {k: list(v) for k, v in data_stream_schemas.items()}
        self.options = L.default_options(**options)
        err = C.create_string_buffer(1024)
        h = self._lib.cep_operator_create(C.byref(self.options), err, len(err))
        if not h:
            L.raise_for(L.CEP_E_DEVICE, err.value.decode())
        self._h = C.c_void_p(h)
        self._views: Dict[str, SiddhiAppRuntime] = {}
        self._callbacks: Dict[str, Dict[str, Tuple[Optional[Callable], bool]]] = {}
        # the router's executionPlanIdToPartitionKeys (AddRouteOperator.java:43,
        # :159-175): appended on add and on update, dropped on delete
        self._partition_keys: Dict[str, List[str]] = {}
        self._inputs: Dict[str, List[str]] = {}    # inputStreamToExecutionPlans, inverted
        self._enabled: Dict[str, bool] = {}        # executionPlanEnabled

    # -- lifecycle -----------------------------------------------------------
    def shutdown(self):
        if self._h:
            self._lib.cep_operator_destroy(self._h)
            self._h = None
            self._views.clear()

    def __del__(self):
        try:
            self.shutdown()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != L.CEP_OK:
            L.raise_for(rc, self._lib.cep_operator_last_error(self._h).decode())

    # -- plans -----------------------------------------------------------------
    def enriched_plan(self, plan: str) -> str:
        """SiddhiExecutionPlanner.getEnrichedExecutionPlan: data stream
        definitions + the plan text."""
        return "".join(stream_definition_expression(s, a) for s, a in self.schemas.items()) + plan

    def _input_streams(self, plan: str) -> List[str]:
        return plan_input_streams(self.enriched_plan(plan))

    def _add_keys(self, plan_id: str, plan: str):
        keys = self._partition_keys.setdefault(plan_id, [])
        full = self.enriched_plan(plan)
        streams = self._input_streams(plan)
        self._inputs[plan_id] = streams
        for s in streams:
            keys.extend(plan_partition_keys(full, s))

    def _view(self, plan_id: str) -> SiddhiAppRuntime:
        h = self._lib.cep_operator_plan(self._h, plan_id.encode())
        if not h:
            raise KeyError(plan_id)
        v = SiddhiAppRuntime._borrow(h, self.options)
        for out_id, (fn, copy) in self._callbacks.get(plan_id, {}).items():
            try:
                v.stream_definition(out_id)
            except L.SiddhiError:
                continue   # the updated plan no longer produces out_id
            v.add_callback(out_id, fn, copy=copy)
        return v

    def add_plan(self, plan_id: str, plan: str):
        self._check(self._lib.cep_operator_add_plan(self._h, plan_id.encode(),
                                                     self.enriched_plan(plan).encode()))
        self._views[plan_id] = self._view(plan_id)
        self._add_keys(plan_id, plan)
        self._enabled[plan_id] = True

    def update_plan(self, plan_id: str, plan: str):
        old = self._views.get(plan_id)   # its callbacks run while the old runtime flushes
        self._check(self._lib.cep_operator_update_plan(self._h, plan_id.encode(),
                                                        self.enriched_plan(plan).encode()))
        new = self._view(plan_id)
        if old is not None:
            old._h = None
            for out_id, rows in old._collected.items():   # rows the old runtime emitted
                if rows:
                    new._collected.setdefault(out_id, [])[:0] = rows
        self._views[plan_id] = new
        self._add_keys(plan_id, plan)

    def remove_plan(self, plan_id: str):
        self._check(self._lib.cep_operator_remove_plan(self._h, plan_id.encode()))
        v = self._views.pop(plan_id, None)
        if v is not None:
            v._h = None
        self._callbacks.pop(plan_id, None)
        self._partition_keys.pop(plan_id, None)
        self._inputs.pop(plan_id, None)
        self._enabled.pop(plan_id, None)

    def enable(self, plan_id: str, enabled: bool = True):
        self._check(self._lib.cep_operator_enable(self._h, plan_id.encode(), 1 if enabled else 0))
        if plan_id in self._enabled:
            self._enabled[plan_id] = bool(enabled)

    def intern(self, s: str) -> int:
        """Id of `s` in the plans' shared string dictionary (STRING columns)."""
        return self._lib.cep_operator_intern(self._h, s.encode())

    def lookup(self, i: int) -> Optional[str]:
        r = self._lib.cep_operator_lookup(self._h, int(i))
        return None if r is None else r.decode()

    def plan_ids(self) -> List[str]:
        buf = C.create_string_buffer(1 << 16)
        self._check(self._lib.cep_operator_plan_ids(self._h, buf, len(buf)))
        v = buf.value.decode()
        return v.split("\n") if v else []

    def plan(self, plan_id: str) -> SiddhiAppRuntime:
        """The plan's runtime (stats, snapshot, output_tensors)."""
        return self._views[plan_id]

    def partition_keys(self, plan_id: str) -> List[str]:
        return list(self._partition_keys.get(plan_id, []))

    def on_event_received(self, event: ControlEvent):
        """AbstractSiddhiOperator.onEventReceived (:400-467)."""
        if isinstance(event, MetadataControlEvent):
            for pid in event.deleted:
                self.remove_plan(pid)
            for pid, plan in event.added.items():
                self.add_plan(pid, plan)
            for pid, plan in event.updated.items():
                self.update_plan(pid, plan)
        elif isinstance(event, OperationControlEvent):
            if event.action is None:
                return
            if event.action == OperationControlEvent.Action.ENABLE_QUERY:
                self.enable(event.query_id, True)
            elif event.action == OperationControlEvent.Action.DISABLE_QUERY:
                self.enable(event.query_id, False)
            else:
                raise ValueError("Illegal action type %s" % event.action)
        else:
            raise ValueError("Illegal event type %r" % (event,))

    # -- output ----------------------------------------------------------------
    def add_callback(self, plan_id: str, out_id: str,
                     fn: Optional[Callable[[OutputRows], None]] = None, copy: bool = True):
        """A StreamCallback on one plan's output stream; kept across updates of
        the plan while the new plan still defines out_id."""
        self._callbacks.setdefault(plan_id, {})[out_id] = (fn, copy)
        self._views[plan_id].add_callback(out_id, fn, copy=copy)

    def collect(self, plan_id: str, out_id: str) -> OutputRows:
        return self._views[plan_id].collect(out_id)

    # -- input -----------------------------------------------------------------
    def process(self, stream_id: str, ts, cols: Sequence) -> int:
        """A batch of stream_id's records to every enabled plan reading it
        (AddRouteOperator.java:65-96); returns the number of plans reached."""
        if stream_id not in self.schemas:
            raise L.UndefinedStreamException("Input stream: %s is not defined" % stream_id)
        types = [t for _, t in self.schemas[stream_id]]
        on_device = _is_device(ts)
        keep = []
        ptrs = (C.c_void_p * max(1, len(cols)))()
        for i, c in enumerate(cols):
            want = np.dtype(L.NUMPY_DTYPES[_TYPE_IDS[types[i]]]) if i < len(types) else None
            p, k = _ptr(c, want, on_device)
            ptrs[i] = p
            keep.append(k)
        tsp, k = _ptr(ts, np.dtype("int64"), on_device)
        keep.append(k)
        b = L.cep_batch(n=_len(ts), ts=tsp, stream=None, input=0, ncols=len(cols),
                        cols=ptrs, on_device=1 if on_device else 0)
        views = list(self._views.values())
        if on_device:
            for v in views:
                v._wait_producer(ts)
        sent = C.c_int(0)
        self._check(self._lib.cep_operator_send(self._h, stream_id.encode(), C.byref(b),
                                                C.byref(sent)))
        if on_device:
            for v in views:
                v._signal_consumer(ts)
        return sent.value

    def flush(self):
        self._check(self._lib.cep_operator_flush(self._h))

    def route(self, stream_id: str, ts, cols: Sequence, nchan: int, seq0: int = 0,
              keys: bool = False) -> Dict[str, object]:
        """AddRouteOperator + DynamicPartitioner for a device batch: plan id ->
        int32 channel per row (and int64 partition key with keys=True) for
        every enabled plan reading stream_id.  The key is the plan's last
        partition key (AddRouteOperator.java:83-92 overwrites it per key);
        a plan without group-by keys gets -1 and a pseudo-random channel."""
        out = {}
        for pid, v in self._views.items():
            if not self._enabled.get(pid) or stream_id not in self._inputs.get(pid, ()):
                continue
            pk = self._partition_keys.get(pid, [])
            out[pid] = v.partition_channels(stream_id, ts, cols, pk[-1] if pk else None,
                                            nchan, seq0, keys=keys)
        return out


_TYPE_IDS = {"int": L.INT, "long": L.LONG, "float": L.FLOAT, "double": L.DOUBLE,
             "bool": L.BOOL, "string": L.STRING}
