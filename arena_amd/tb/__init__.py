"""TensorBoard-compatible scalar logging (tfevents writer/reader) and a built-in viewer."""
from .writer import SummaryWriter, read_scalars  # noqa: F401
