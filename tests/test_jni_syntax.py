"""CPU: the JNI glue (java/jni/hbam_jni.c) type-checks.

No JDK exists in this image, so `gcc -fsyntax-only` runs the glue against
tests/jni_min/jni.h, a minimal header written from the JNI specification (the
C types and the function-table entries the glue calls), and the real
include/hbam.h.  Every JNIEnv / JavaVM call is checked for its argument count
and types, every hbam_* call against the C ABI's prototypes; warnings are
errors."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "java", "jni", "hbam_jni.c")
STUB = os.path.join(ROOT, "tests", "jni_min")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not installed")
def test_jni_glue_compiles_against_the_jni_specification():
    r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Wall", "-Wextra", "-Wno-unused-parameter",
                        "-Werror", "-I", STUB, "-I", os.path.join(ROOT, "include"), JNI],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_stub_declares_every_table_entry_the_glue_calls():
    src = open(JNI).read()
    stub = open(os.path.join(STUB, "jni.h")).read()
    called = set(re.findall(r"\(\*(?:env|r->vm|\(JavaVM \*\)vm)\)->(\w+)", src))
    assert len(called) >= 25
    declared = set(re.findall(r"\(JNICALL \*(\w+)\)", stub))
    assert called <= declared, called - declared
