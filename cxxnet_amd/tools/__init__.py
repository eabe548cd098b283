"""Data-preparation tools (reference tools/): im2bin and the imgbin partition maker."""
