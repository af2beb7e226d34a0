from veles_amd.models.zoo import lenet

root.common.engine.precision_type = "bfloat16"  # noqa: F821 (root is injected)
root.mnist_conv.update({  # noqa: F821
    "loader_name": "synthetic_images",
    "loader": {"dataset": "mnist", "class_lengths": (1000, 1000, 6000),
               "minibatch_size": 100, "normalization_type": "mean_disp",
               "noise": 110.0},
    "decision": {"max_epochs": 10, "fail_iterations": 20},
    "snapshotter": {"prefix": "mnist_conv", "interval": 1,
                    "time_interval": 0},
})
root.mnist_conv.layers = lenet()  # noqa: F821
