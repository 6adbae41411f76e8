"""microrts_amd — MI355X-native vectorised microRTS env step (HIP kernels behind a C ABI).

Drop-in for tests.JNIGridnetVecClient of the reference (src/tests/JNIGridnetVecClient.java).
"""
from .vec_client import JNIGridnetVecClient, UnitTypeTable, DeviceVecEnv, ForwardModel  # noqa: F401

__all__ = ["JNIGridnetVecClient", "UnitTypeTable", "DeviceVecEnv", "ForwardModel"]
