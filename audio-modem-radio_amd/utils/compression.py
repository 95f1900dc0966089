"""Import path of the reference (`from utils.compression import ...`, decoder.py:15)."""
from compression import (IntelligentCompressor, adaptive_compress, compress_data, decompress_data,  # noqa: F401
                         delta_compress, delta_decompress, intelligent_compress, intelligent_decompress,
                         super_compress, super_decompress, prepare_sstv_like)
