"""Probe: what amdsmi reports per process (pid, VRAM) for a child that holds
1 GiB of HBM, next to the child's own pid and the device's vram_used."""
import json
import os
import subprocess
import sys
import time

CHILD = ('import torch,time,os;x=torch.empty(1<<30,dtype=torch.uint8,'
         'device="cuda");torch.cuda.synchronize();print(os.getpid(),'
         'flush=True);time.sleep(20)')


def main():
    child = subprocess.Popen([sys.executable, '-c', CHILD],
                             stdout=subprocess.PIPE, text=True)
    pid = int(child.stdout.readline())
    import amdsmi
    amdsmi.amdsmi_init()
    out = {'child_pid': pid, 'self_pid': os.getpid(), 'devices': []}
    for handle in amdsmi.amdsmi_get_processor_handles():
        dev = {'bdf': str(amdsmi.amdsmi_get_gpu_device_bdf(handle))}
        try:
            dev['vram'] = amdsmi.amdsmi_get_gpu_vram_usage(handle)
        except Exception as err:  # pylint: disable=broad-except
            dev['vram_error'] = repr(err)
        try:
            dev['procs'] = amdsmi.amdsmi_get_gpu_process_list(handle)
        except Exception as err:  # pylint: disable=broad-except
            dev['procs_error'] = repr(err)
        try:
            dev['compute_procs'] = [
                str(p) for p in amdsmi.amdsmi_get_gpu_compute_process_info()]
        except Exception as err:  # pylint: disable=broad-except
            dev['compute_procs_error'] = repr(err)
        out['devices'].append(dev)
    child.kill()
    child.wait()
    print(json.dumps(out, default=str, indent=1))
    amdsmi.amdsmi_shut_down()
    time.sleep(0)


if __name__ == '__main__':
    main()
