"""horreum_amd — MI355X-native SSTable record codec for ikanago/horreum.

The product is libhorreum_gpu.so (C ABI: include/horreum_gpu.h; HIP kernels
for gfx950 in horreum_amd/csrc).  This package is its Python host side:

- ``abi``     ctypes binding of the C ABI (raises if the library is missing);
- ``engine``  device/host buffers around the ABI (torch for HBM and streams);
- ``format``  mirror of the reference's src/format.rs API (InternalPair ...);
- ``index``, ``storage``, ``table``  mirrors of src/sstable/{index,storage,table}.rs.
"""
from .abi import HorreumGpuError, Status  # noqa: F401

__all__ = ["HorreumGpuError", "Status"]
