"""A `torch_xla`-API adapter for the MI355X build.

train_DSTAGNN_my.py hard-imports torch_xla (:17-18, :196) and drives its device, optimiser step,
loaders and process spawning through it (:25, :33, :113-115, :127, :148-161, :173-183, :195-197).
With `dstagnn_drought_amd.refpaths.install()` on sys.path these imports resolve here and map onto
the HIP device and torch.distributed (RCCL, backend "nccl"):

    xm.xla_device()            -> cuda:<LOCAL_RANK> (process group initialised when WORLD_SIZE > 1)
    xm.optimizer_step(opt)     -> GradAllReducer.all_reduce() (mean over ranks) + opt.step()
    xm.xrt_world_size / get_ordinal / is_master_ordinal / master_print / get_memory_info / save
    pl.MpDeviceLoader(loader)  -> the loader's batches copied to the device
    xmp.spawn(fn, nprocs=n)    -> n processes, one GPU each, torch.distributed env set

This is plumbing, not compute: every tensor op of the model runs in libdstagnn.so."""
__version__ = "2.0+dstagnn_mi355x"
