#!/usr/bin/env python3
"""Print an ENAS child nn_config (enas suggestion output format) whose op ids 0..5 cover
conv / separable (dm 2) / depthwise (7x7 s2, 3x3 dm 2) / strided conv / max pool."""
import json

emb = {
    "0": {"opt_id": 0, "opt_type": "convolution", "filter_size": "3", "num_filter": "32", "stride": "1"},
    "1": {"opt_id": 1, "opt_type": "separable_convolution", "filter_size": "5", "num_filter": "48", "stride": "1",
          "depth_multiplier": "2"},
    "2": {"opt_id": 2, "opt_type": "depthwise_convolution", "filter_size": "7", "stride": "2", "depth_multiplier": "1"},
    "3": {"opt_id": 3, "opt_type": "depthwise_convolution", "filter_size": "3", "stride": "1", "depth_multiplier": "2"},
    "4": {"opt_id": 4, "opt_type": "convolution", "filter_size": "5", "num_filter": "64", "stride": "2"},
    "5": {"opt_id": 5, "opt_type": "reduction", "reduction_type": "max_pooling", "pool_size": 2},
}
print(json.dumps({"num_layers": 6, "input_sizes": [32, 32, 3], "output_sizes": [10], "embedding": emb}))
