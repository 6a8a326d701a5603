"""gcslam — MI355X-native GC-SLAM v2 per-scan hot path (Python host over a HIP C-ABI)."""
