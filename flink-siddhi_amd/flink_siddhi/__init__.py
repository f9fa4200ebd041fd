"""flink_siddhi — MI355X-native CEP matching engine (Python host side).

Python mirror of the flink-siddhi surface over libcep.so's C ABI:
  * `runtime.SiddhiAppRuntime` — the Siddhi app-runtime calls the operator
    makes (AbstractSiddhiOperator.java:114-176): send / process_elements /
    process_watermark (event-time reorder, :222-247), callbacks, snapshot,
  * `operator.SiddhiOperator` — dynamic plans driven by control events
    (onEventReceived, :400-467; router/AddRouteOperator.java),
  * `shuffle` — the multi-GPU key shuffle (router/HashPartitioner.java),
  * `workload` — the BASELINE synthetic streams.
"""
from ._lib import (CepCapacityError, CepDeviceError, CepStateError,  # noqa: F401
                   DuplicatedStreamException, SiddhiAppCreationException,
                   SiddhiError, UndefinedStreamException,
                   UnsupportedPlanException)
from .runtime import SiddhiAppRuntime, plan_schema, validate  # noqa: F401
from .operator import (MetadataControlEvent, OperationControlEvent,  # noqa: F401
                       SiddhiOperator)
