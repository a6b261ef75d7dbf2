"""Per-kernel resources from a device assembly file's amdhsa.kernels metadata:
    python tools/kernel_resources.py file.s [name-substring]"""
import re
import sys

import yaml


def main():
    s = open(sys.argv[1]).read()
    m = re.search(r"\.amdgpu_metadata\n(.*?)\.end_amdgpu_metadata", s, re.S)
    meta = yaml.safe_load(m.group(1).replace("\t", "    "))
    for k in meta["amdhsa.kernels"]:
        if len(sys.argv) > 2 and sys.argv[2] not in k[".name"]:
            continue
        print(f'{k[".name"][:70]:70s} vgpr {k[".vgpr_count"]:3d} agpr {k.get(".agpr_count", 0):3d} '
              f'sgpr {k[".sgpr_count"]:3d} spill {k[".vgpr_spill_count"]} lds {k[".group_segment_fixed_size"]} '
              f'scratch {k[".private_segment_fixed_size"]}')


if __name__ == "__main__":
    main()
