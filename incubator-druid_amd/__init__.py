"""MI355X-native segment scan-and-aggregate engine for Druid segments (timeseries / topN / groupBy).

Import with ``importlib.import_module("incubator-druid_amd")`` (the directory name carries a hyphen).
"""
