"""Stand-in for isaacgym.gymutil (only what the reference's env construction path calls)."""


def parse_device_str(device_str):
    # isaacgym.gymutil.parse_device_str: 'cuda:0' -> ('cuda', 0); 'cpu' -> ('cpu', 0)
    if device_str == "cpu" or device_str.startswith("cpu"):
        return "cpu", 0
    if ":" in device_str:
        t, i = device_str.split(":")
        return t, int(i)
    return device_str, 0
