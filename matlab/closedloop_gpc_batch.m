function [J, F, status, traj] = closedloop_gpc_batch(sc, N, Nu, delta, lambda, opts)
% CLOSEDLOOP_GPC_BATCH  The batched entry of SURVEY §8b: C candidates in one GPU call.
%   sc        struct: h = mpct_mex('create', mpct_scenario_from_mpc(...)) handle, r (my x nit,
%             Par.Xsp), v (nd x nit, Par.mdv, [] if none), my, nu; optional devices (GPU list:
%             mpct_mex('eval_multi') shards the candidates over them)
%   N, Nu     C x 1 horizons (max(N), max(Nu) per candidate, closedloop_toolbox.m:38-40)
%   delta     C x my Weights.OV,  lambda  C x nu Weights.MVRate
%   opts      struct: vns (1: the VNS2.m:147-195 objective), want_traj
% Returns J (C x my): GAM_fun.m:110-111 J1 per output; F (C x 1): the VNS objective
% sum(j21 + j22) + N(1) + sum(Jnu) (square plants: one unit-step simulation per output, output
% and MV i from simulation i, VNS2.m:148-165; non-square: one simulation with every output
% stepped at inK, VNS2.m:166-169), NaN where a simulation failed; status (C x nref); traj: y, u,
% ys, uopt of every simulation (my x nit x S) when opts.want_traj.
if nargin < 6, opts = struct(); end
vns = isfield(opts, 'vns') && opts.vns;
C = numel(N); my = sc.my; nu = sc.nu; nit = size(sc.r, 2);
if vns
    inK = 10;
    if my == nu
        R = zeros(my, nit, my);
        for i = 1:my, R(i, inK:end, i) = 1; end      % Xsp.*sel, VNS2.m:58-61,148-150
    else
        R = zeros(my, nit); R(:, inK:end) = 1;         % Xsp, VNS2.m:168
    end
else
    R = sc.r;
end
o = struct('open_loop', double(vns), 'want_traj', double(isfield(opts, 'want_traj') && opts.want_traj));
if isfield(sc, 'devices') && numel(sc.devices) > 1
    [J1, j21, j22, Jnu, st, ~, y, u, ys, uopt] = mpct_mex('eval_multi', sc.h, sc.devices, N(:), Nu(:), ...
                                                          delta, lambda, R, sc.v, o);
else
    [J1, j21, j22, Jnu, st, ~, y, u, ys, uopt] = mpct_mex('eval', sc.h, N(:), Nu(:), delta, lambda, R, sc.v, o);
end
nref = size(R, 3);
status = reshape(st, nref, C).';
bad = any(bitand(status, 2 + 4 + 8 + 16 + 128), 2);
J = J1(1:nref:end, :);
F = nan(C, 1);
if vns
    if my == nu                                         % output / MV i from simulation i
        idx = (0:C-1)' * nref;
        a21 = zeros(C, my); a22 = zeros(C, my); anu = zeros(C, nu);
        for i = 1:my
            a21(:, i) = j21(idx + i, i); a22(:, i) = j22(idx + i, i); anu(:, i) = Jnu(idx + i, i);
        end
    else
        a21 = j21; a22 = j22; anu = Jnu;
    end
    F = sum(a21 + a22, 2) + N(:) + sum(anu, 2);
end
F(bad) = NaN;
J(bad, :) = NaN;
traj = struct('y', y, 'u', u, 'ys', ys, 'uopt', uopt);
end
