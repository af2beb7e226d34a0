from veles_amd.models.zoo import cifar_quick

root.common.engine.precision_type = "bfloat16"  # noqa: F821 (root is injected)
root.cifar_conv.update({  # noqa: F821
    "loader_name": "synthetic_images",
    "loader": {"dataset": "cifar10", "class_lengths": (1000, 1000, 8000),
               "minibatch_size": 100, "normalization_type": "mean_disp",
               "noise": 110.0},
    "decision": {"max_epochs": 10, "fail_iterations": 20},
    "snapshotter": {"prefix": "cifar_conv", "interval": 1,
                    "time_interval": 0},
})
root.cifar_conv.layers = cifar_quick()  # noqa: F821
