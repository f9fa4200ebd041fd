"""flink_siddhi — MI355X-native CEP matching engine (Python host side).

Python mirror of the flink-siddhi surface over libcep.so's C ABI:
  * `runtime.SiddhiAppRuntime` — the Siddhi app-runtime calls the operator
    makes (AbstractSiddhiOperator.java:114-176),
  * `operator.SiddhiStreamOperator` — the operator shell (event-time reorder
    queue, watermark drain, snapshot) of AbstractSiddhiOperator.java:92-468,
  * `cep.SiddhiCEP` / `SiddhiStream` — the user DSL (SiddhiCEP.java,
    SiddhiStream.java) driving a local event-time job.
"""
from ._lib import (CepCapacityError, CepDeviceError, CepStateError,  # noqa: F401
                   DuplicatedStreamException, SiddhiAppCreationException,
                   SiddhiError, UndefinedStreamException,
                   UnsupportedPlanException)
from .runtime import SiddhiAppRuntime, plan_schema, validate  # noqa: F401
