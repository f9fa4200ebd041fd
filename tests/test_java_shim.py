"""CPU: the Java operator shim and its JNI layer agree with each other and
with include/cep.h (no JDK exists in this image, so the shim ships as source:
flink-siddhi_amd/java/.../gpu/*.java, flink-siddhi_amd/jni/cep_jni.c).

Checked here: every `native` method of CepNative.java has exactly one JNI
implementation with the mangled name; every libcep function the JNI layer
calls is declared in include/cep.h and exported by libcep.so."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
JAVA = ROOT / "flink-siddhi_amd" / "java" / "org" / "apache" / "flink" / "streaming" / "siddhi" / "gpu"
JNI = ROOT / "flink-siddhi_amd" / "jni" / "cep_jni.c"
HDR = ROOT / "include" / "cep.h"
LIB = ROOT / "flink-siddhi_amd" / "libcep.so"


def _natives():
    src = (JAVA / "CepNative.java").read_text()
    return re.findall(r"static native [\w\[\]<>.]+ (\w+)\(", src)


def test_every_native_method_has_one_jni_implementation():
    natives = _natives()
    assert len(natives) == len(set(natives)) > 10
    impl = re.findall(r"JNICALL FN\((\w+)\)", JNI.read_text())
    assert sorted(impl) == sorted(natives)


def test_jni_calls_only_declared_and_exported_cep_functions():
    declared = set(re.findall(r"\b(cep_\w+)\s*\(", HDR.read_text()))
    called = set(re.findall(r"\b(cep_\w+)\s*\(", JNI.read_text()))
    assert called, "the JNI layer calls libcep"
    assert called <= declared, called - declared
    if not LIB.exists():
        pytest.skip("libcep.so not built")
    lib = ctypes.CDLL(str(LIB))
    for name in sorted(called):
        assert hasattr(lib, name), name


def test_operator_shim_covers_the_reference_operator_hooks():
    src = (JAVA / "GpuSiddhiStreamOperator.java").read_text()
    # the reference operator's entry points (AbstractSiddhiOperator.java) the shim replaces
    for hook in ("processElement", "processWatermark", "snapshotState", "initializeState", "open", "close",
                 "onEventReceived", "prepareSnapshotPreBarrier"):
        assert re.search(r"public void %s\(" % hook, src), hook
    for state in ('"siddhiRuntimeState"', '"queuedRecordsState"'):
        assert state in src
