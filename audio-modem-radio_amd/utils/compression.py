"""Import path of the reference (`from utils.compression import ...`, decoder.py:15)."""
from compression import delta_compress, delta_decompress, intelligent_decompress  # noqa: F401
