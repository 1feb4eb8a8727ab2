"""Which backend do DeviceMesh sub-groups get when the default process group
is gloo and the mesh device type is cuda (4 ranks sharing cuda:0)?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hipsnapshot.utils.test_utils import run_distributed  # noqa: E402


def w():
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import Shard, distribute_tensor

    torch.cuda.set_device(0)
    for names in (("dp", "tp"), ("tp", "dp")):
        mesh = init_device_mesh("cuda", (2, 2), mesh_dim_names=names)
        for n in names:
            g = mesh[n].get_group()
            print(dist.get_rank(), names, n, dist.get_backend(g), flush=True)
        x = distribute_tensor(torch.arange(16.0, device="cuda").view(4, 4), mesh,
                              [Shard(0), Shard(1)])
        print(dist.get_rank(), names, "full ok", bool((x.full_tensor().cpu() ==
                                                       torch.arange(16.0).view(4, 4)).all()),
              flush=True)


if __name__ == "__main__":
    run_distributed(w, 4, timeout=120)
