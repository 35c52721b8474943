"""s3dlio_amd — MI355X-native synthetic object-payload generator.

Drop-in for s3dlio's data-generation hot path (src/data_gen.rs), built as
hand-written gfx950 HIP kernels behind a C ABI (include/s3dlio_gpu.h,
libs3dlio_amd.so).  Importing this package loads the library; it raises if
the library is absent (no CPU fallback exists).
"""
from ._lib import S3dgError, lib  # noqa: F401  (loads libs3dlio_amd.so)
from .hostbuf import BytesView  # noqa: F401
from .device import (BLOCK_SIZE, DEFAULT_BASE_SEED, Context, compress_ratio,  # noqa: F401
                     device_count, host_context, host_slots, object_entropy, parse_devices,
                     unique_blocks, xoshiro_jump)
from .data_gen import (HostRegistration, fill_controlled_data, fill_controlled_data_seeded,  # noqa: F401
                       register_host_buffer, unregister_host_buffer)
from .datagen import (DataGenerator, Generator, ObjectGen, default_data_gen_threads,  # noqa: F401
                      generate_controlled_data_alt, generate_controlled_data_streaming,
                      generate_data, generate_data_with_threads, generate_into_buffer,
                      optimal_chunk_size, py_default_data_gen_threads, py_total_cpus,
                      total_cpus, NumaMode, GeneratorConfig, DataBuffer, ObjectGenAlt,
                      generate_data_from_config, generate_data_simple, generate_data_with_config)

from .npz import crc32_combine, crc32_device, generate_npz_bytes, npz_size  # noqa: F401

from .objects import (Config, DataGenMode, ObjectType, build_npz, build_raw,  # noqa: F401
                      build_tfrecord, build_tfrecord_with_index, generate_object,
                      generate_random_data, object_size)

from .put import (DEFAULT_OBJECT_SIZE, PutResult, build_uri_list, put,  # noqa: F401
                  put_objects, put_objects_with_random_data_and_type)

__version__ = "0.1.0"
