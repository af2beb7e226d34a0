from veles_amd.models.zoo import vgg16

root.common.engine.precision_type = "float8"  # noqa: F821 (root is injected)
root.vgg16.update({  # noqa: F821
    "loader_name": "synthetic_images",
    "loader": {"dataset": "imagenet224", "class_lengths": (0, 256, 4096),
               "minibatch_size": 128, "normalization_type": "mean_disp",
               "noise": 110.0},
    "decision": {"max_epochs": 2, "fail_iterations": 20},
    "snapshotter": {"prefix": "vgg16", "interval": 1,
                    "time_interval": 0},
})
root.vgg16.layers = vgg16()  # noqa: F821
