from veles_amd.models.zoo import alexnet

root.common.engine.precision_type = "bfloat16"  # noqa: F821 (root is injected)
root.alexnet.update({  # noqa: F821
    "loader_name": "synthetic_images",
    "loader": {"dataset": "imagenet", "class_lengths": (0, 512, 8192),
               "minibatch_size": 256, "normalization_type": "mean_disp",
               "noise": 110.0},
    "decision": {"max_epochs": 2, "fail_iterations": 20},
    "snapshotter": {"prefix": "alexnet", "interval": 1,
                    "time_interval": 0},
})
root.alexnet.layers = alexnet()  # noqa: F821
