from veles_amd.models.zoo import mnist_fc

root.mnist_fc.update({  # noqa: F821 (root is injected)
    "loader_name": "synthetic_images",
    "loader": {"dataset": "mnist", "class_lengths": (1000, 1000, 6000),
               "minibatch_size": 100, "normalization_type": "mean_disp",
               "noise": 110.0},
    "layers": {"dict": True, "v": mnist_fc()},
    "decision": {"max_epochs": 5, "fail_iterations": 20},
    "snapshotter": {"prefix": "mnist_fc", "interval": 1,
                    "time_interval": 0},
})
root.mnist_fc.layers = mnist_fc()  # noqa: F821
