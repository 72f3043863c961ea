function [y,u,yopt,uopt] = closedloop_toolbox_nmpc(nmpcobj,model,init,r,N,Nu,delta,lambda,nit)
% CLOSEDLOOP_TOOLBOX_NMPC  Drop-in for Matlab-Toolbox/NMPC/closedloop_toolbox_nmpc.m:1 (callers
% VNS2.m:155, GAM_fun.m:87, VanDeVusse_NMPC.m:244) on the MI355X engine.  A C ABI cannot carry a
% MATLAB function handle to the GPU, so the model is recognised by name: the Van de Vusse reactor
% of nmpc_vandevusse_state.m (MPCT_NMPC_VANDEVUSSE, its parameters built in); other models error.
% Bounds come from nmpcobj.MV / States, ScaleFactors from nmpcobj.OV / MV, Ts from nmpcobj.Ts,
% x0 / u0 / output states from init (init.x0, init.u0, init.xc).  The prediction and the plant
% use fixed-step RK4 with 10 sub-steps per Ts (DESIGN.md §12; nlmpc's fmincon / ode15s are closed
% source).
persistent cache
name = func2str(model);
assert(contains(lower(name), 'vandevusse'), 'mpct:nmpc', ...
       'only the Van de Vusse model (nmpc_vandevusse_state.m) is built into libmpct, got %s', name);
if size(r, 1) > size(r, 2), r = r.'; end
ny = numel(init.xc); nx = numel(init.x0); nu = numel(init.u0);
key = {init.x0(:).', init.u0(:).', init.xc(:).', [nmpcobj.MV.Min], [nmpcobj.MV.Max], ...
       [nmpcobj.States.Min], [nmpcobj.States.Max], [nmpcobj.OV.ScaleFactor], [nmpcobj.MV.ScaleFactor], ...
       nmpcobj.Ts, nit};
n2 = max(N); nuh = max(Nu);
if isempty(cache) || ~isequal(cache.key, key) || n2 > cache.n_max || nuh > cache.nu_max
    if ~isempty(cache), mpct_mex('destroy', cache.h); end
    d = struct('model', 1, 'nx', nx, 'ny', ny, 'nu', nu, 'xc', init.xc(:).', 'ts', nmpcobj.Ts, 'nsub', 10, ...
               'x0', init.x0(:).', 'u0', init.u0(:).', 'u_min', [nmpcobj.MV.Min], 'u_max', [nmpcobj.MV.Max], ...
               'x_min', [nmpcobj.States.Min], 'x_max', [nmpcobj.States.Max], ...
               'y_scale', [nmpcobj.OV.ScaleFactor], 'u_scale', [nmpcobj.MV.ScaleFactor], ...
               'n_max', max(n2, 31), 'nu_max', min(max(nuh, 15), floor(32 / nu)), 'nit', nit, ...
               'yref', zeros(ny, nit), 'vns_ink', 10);
    cache = struct('key', {key}, 'h', mpct_mex('create_nmpc', d), 'n_max', d.n_max, 'nu_max', d.nu_max);
end
opts = struct('open_loop', 1, 'want_traj', 1);
[~,~,~,~,status,~,y,u,yopt,uopt] = mpct_mex('eval', cache.h, n2, nuh, delta(:).', lambda(:).', ...
                                            r(:, 1:nit), [], opts);
if bitand(status, 2 + 4 + 8 + 16 + 128)
    error('mpct:nlmpc', 'closed-loop NMPC simulation failed (status %d)', status);
end
end
