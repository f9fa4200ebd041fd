"""C-ABI checks that need no GPU: libcep.so loads, exports every entry point
include/cep.h declares, the Python binding covers them, and the host-side
front end (validate / plan_schema — SiddhiManager.validateSiddhiApp,
AbstractSiddhiOperator.java:292-299) runs without a device.  The product path
itself fails loudly when no GPU is present (no CPU fallback)."""
import ctypes
import re
from pathlib import Path

import pytest

import flink_siddhi as fs
from flink_siddhi import _lib as L
from flink_siddhi import workload

HEADER = Path(__file__).resolve().parents[1] / "include" / "cep.h"


def header_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(cep_[a-z_0-9]+)\s*\(", text))
    # typedef'd callback type is not a function
    names.discard("cep_emit_fn")
    return sorted(names)


def test_header_declares_the_boundary():
    names = header_functions()
    for must in ("cep_create", "cep_send_batch", "cep_flush", "cep_snapshot",
                 "cep_restore", "cep_validate", "cep_destroy"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(str(L.LIB_PATH))
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_every_declared_symbol():
    missing = [n for n in header_functions() if n not in L.SIGNATURES]
    assert not missing, missing


def test_validate_and_schema_on_host():
    fs.validate(workload.PATTERN_PLAN)
    attrs = fs.plan_schema(workload.PATTERN_PLAN, "O")
    assert [a[0] for a in attrs] == ["k", "p1", "p2", "t"]
    with pytest.raises(fs.SiddhiAppCreationException):
        fs.validate("define stream A (x int); from A[x >] select x insert into O;")
    with pytest.raises(fs.UndefinedStreamException):
        fs.validate("define stream A (x int); from B select x insert into O;")


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(fs.CepDeviceError):
        fs.SiddhiAppRuntime(workload.PATTERN_PLAN)
