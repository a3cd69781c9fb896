"""The JNI adaptor (scenery-insitu_amd/jni/insitu_jni.cpp) compiles against the C ABI it binds: a
syntax-only g++ pass with tests/jni_stub/jni.h standing in for the JDK header this image lacks (the
real build needs JAVA_HOME).  Catches drift between the adaptor and include/insitu_hip.h."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_jni_adaptor_compiles_against_the_c_abi():
    p = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
                        f"-I{ROOT / 'tests' / 'jni_stub'}", f"-I{ROOT / 'include'}",
                        f"-I{ROOT / 'scenery-insitu_amd' / 'jni'}", str(ROOT / "scenery-insitu_amd" / "jni" / "insitu_jni.cpp")],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-4000:]
