// Host-native (CPU) layer of the framework: libsq_host, loaded with ctypes
// by ``sq_learn_amd/ops/_host.py``.  Plain extern "C" entry points taking raw
// pointers and sizes; OpenMP for row/source parallelism (the reference's
// own intra-op model).  No HIP, no CPython API: it builds and
// runs on any host, including CPU-only test machines.
#pragma once
#include <algorithm>
#include <cstdint>
