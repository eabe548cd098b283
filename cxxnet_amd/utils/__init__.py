"""Utilities: evaluation metrics (utils.metric: host MetricSet over the native C++ metrics and
the device-side DeviceMetricSet).  The config reader is native (csrc/runtime/config_reader.h,
exposed through cxxnet_amd.native.rt()) and the step timers are HIP events in the trainer."""
