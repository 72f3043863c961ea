function [y,u,t,ys,uopt] = closedloop_toolbox(mpc_toolbox,r,v,N,Nu,delta,lambda,nit)
% CLOSEDLOOP_TOOLBOX  Drop-in for MPC-Tuning/MPC_Tuning/closedloop_toolbox.m:1 on the MI355X
% engine: same signature, same outputs (row signals y my x nit, u nu x nit, t, ys, uopt), so
% VNS2.m:153,168 and GAM_fun.m:81 run unchanged.  One closed loop of nit steps with
% PredictionHorizon = max(N), ControlHorizon = max(Nu), Weights.OV = delta, Weights.MVRate =
% lambda (:36-43), plus the open-loop first-move prediction uopt / ys (:85-100), all from one
% mpct_mex('eval') call.  Put this folder ahead of MPC_Tuning/ on the MATLAB path.
% The scenario (tables + device copies) is built once per mpc object and horizon range and
% cached; a different object or a larger horizon rebuilds it.
persistent cache
if size(r, 1) > size(r, 2), r = r.'; end            % row2col / col2row: row signals here
if isempty(v), v = zeros(0, nit); elseif size(v, 2) ~= nit, v = v.'; end
Ts = mpc_toolbox.Ts;
key = mpct_cache_key(mpc_toolbox, nit);
n2 = max(N); nuh = max(Nu);
if isempty(cache) || ~isequal(cache.key, key) || n2 > cache.n2_max || nuh > cache.nu_max
    if ~isempty(cache), mpct_mex('destroy', cache.h); end
    n2_max = max(n2, 127); nu_max = max(nuh, 15);
    desc = mpct_scenario_from_mpc(mpc_toolbox, nit, [], n2_max, nu_max);
    nu_max = min(nu_max, floor((63 - isfield(desc, 'mdband')) / desc.nu));  % QP rows fit one wavefront
    desc.nu_max = nu_max;
    cache = struct('key', {key}, 'h', mpct_mex('create', desc), 'n2_max', n2_max, 'nu_max', nu_max);
end
opts = struct('open_loop', 1, 'want_traj', 1);
[~,~,~,~,status,~,y,u,ys,uopt] = mpct_mex('eval', cache.h, n2, nuh, delta(:).', lambda(:).', r(:, 1:nit), ...
                                          v(:, 1:nit), opts);
if bitand(status, 2 + 4 + 8 + 16 + 128)                  % what sim would have thrown (objectives.FATAL_STATUS)
    error('mpct:sim', 'closed-loop simulation failed (status %d)', status);
end
t = (0:nit-1) * Ts;
end

function key = mpct_cache_key(mpcobj, nit)
% everything mpct_scenario_from_mpc reads, so an equal key means an equal scenario
P = tf(mpcobj.Model.Plant);
key = {P.Numerator, P.Denominator, P.IODelay, P.InputGroup, [mpcobj.MV.Min], [mpcobj.MV.Max], ...
       [mpcobj.MV.RateMin], [mpcobj.MV.RateMax], [mpcobj.OV.Min], [mpcobj.OV.Max], [mpcobj.OV.MinECR], ...
       [mpcobj.OV.MaxECR], [mpcobj.OV.ScaleFactor], [mpcobj.MV.ScaleFactor], mpcobj.Weights.ECR, nit};
end
