"""dltb.results — reference-compatible result records, files and stdout markers."""
from .record import (RESULT_KEYS, extract_from_log, make_record, print_markers, print_result,  # noqa: F401
                     result_filename, write_result)
