function desc = mpct_scenario_from_mpc(mpcobj, nit, Yref, n2_max, nu_max)
% MPCT_SCENARIO_FROM_MPC  The candidate-independent part of closedloop_toolbox's inputs as an
% mpct_mex('create', desc) descriptor (include/mpct.h, mpct_scenario_desc, ABI >= 5).
%   mpcobj   the (scaled) toolbox mpc object MPCTuning.m:152-199 builds: Model.Plant = Pze with
%            its MV / MD input groups, MV Min/Max/RateMin/RateMax, OV Min/Max/MinECR/MaxECR,
%            ScaleFactors, Weights.ECR
%   nit      closed-loop length;  Yref  my x nit GAM/VNS reference (Par.Yref), [] = zeros
%   n2_max, nu_max   largest horizons any candidate will use (VNS: 2^nbp-1, 2^nbc-1)
% The plant / model entries are passed as tfdata 'v' rows and IODelay; the library derives the
% CARIMA tables (descompMPC + exact LCM).  Plants with measured disturbances, finite OV bounds or
% non-unit ScaleFactors use the measured-disturbance / soft-band kernel (mdband).
P = tf(mpcobj.Model.Plant);
ig = P.InputGroup;
mv = 1:size(P, 2);
md = [];
if isfield(ig, 'MV'), mv = ig.MV(:)'; end
if isfield(ig, 'MD'), md = ig.MD(:)'; end
P = P(:, [mv md]);                                   % MVs first, then MDs (the ABI's column order)
[my, nin] = size(P);
nu = numel(mv);
nd = numel(md);
[num, den] = tfdata(P, 'v');
if ~iscell(num), num = {num}; den = {den}; end
plant = struct('num', num, 'den', den, 'delay', num2cell(P.IODelay + zeros(my, nin)));
if nargin < 3 || isempty(Yref), Yref = zeros(my, nit); end
if size(Yref, 1) ~= my, Yref = Yref.'; end
MV = mpcobj.MV;
OV = mpcobj.OV;
desc = struct('my', my, 'nu', nu, 'nd', nd, 'nit', nit, 'n2_max', n2_max, 'nu_max', nu_max, ...
              'weights_squared', 1, 'vns_ink', 10, 'n1', ones(1, my), 'plant', plant, ...
              'du_min', [MV.RateMin], 'du_max', [MV.RateMax], 'u_min', [MV.Min], 'u_max', [MV.Max], ...
              'yref', Yref(:, 1:nit));
ymin = [OV.Min]; ymax = [OV.Max];
ysc = [OV.ScaleFactor]; usc = [MV.ScaleFactor];
if nd > 0 || any(isfinite([ymin ymax])) || any(ysc ~= 1) || any(usc ~= 1)
    desc.mdband = 1;
    desc.y_min = ymin;  desc.y_max = ymax;
    desc.ecr_min = [OV.MinECR];  desc.ecr_max = [OV.MaxECR];
    desc.y_scale = ysc;  desc.u_scale = usc;
    desc.rho_ecr = mpcobj.Weights.ECR;
end
end
