"""dltb.data — synthetic token datasets and device-resident batchers."""
from .synthetic import DeviceBatcher, HostBatcher, SyntheticDataset, epoch_indices, make_batcher  # noqa: F401
