"""Data pipeline (reference src/io/)."""
from .data import DataBatch, DataIterator  # noqa: F401
from .iterators import create_iterator  # noqa: F401
