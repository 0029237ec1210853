function [image, views] = renderChannels(renderers, varargin)
% renderChannels  One frame of several VolumeRender objects (channels) in one MEX call.
%
%   image = renderChannels({r1, r2, ...})           % mono: the channels' images summed
%   image = renderChannels({r1, r2, ...}, true)     % stereo pair at r1.CameraXOffset, combined
%   [image, views] = renderChannels(...)            % views: single [H W 3 n*eyes], per channel/eye
%
% examples/example3.m:61-239 renders each channel with its own VolumeRender -- its own volumes,
% colour and factors -- and adds the images; each render is a syncVolumes and one or two 'render'
% calls.  Here every channel's sync and render arguments go to volumeRender('render_channels', ...)
% (vr_render_channels): the channels' views are marched together, and each view equals its own
% syncVolumes + render.  Every channel must have the same ImageResolution.  TimeLastMemSync is
% stamped afterwards, as VolumeRender.syncVolumes does.
stereo = numel(varargin) >= 1 && logical(varargin{1});
n = numel(renderers);
r1 = renderers{1};
base = 0;
resolution = flip(r1.ImageResolution);
delta = 0;
if stereo
    base = r1.CameraXOffset / 2;
    fov = 2 * atan(1 / r1.FocalLength);
    delta = round((base * r1.ImageResolution(2)) / (2 * r1.FocalLength * tan(fov / 2)));
    resolution = resolution + [0, delta];
end
cells = cell(1, n);
for i = 1:n
    r = renderers{i};
    if ~isequal(r.ImageResolution, r1.ImageResolution)
        error('renderChannels: every channel needs the same ImageResolution');
    end
    c = {r.objectHandle, r.TimeLastMemSync, r.VolumeEmission, r.VolumeReflection, r.VolumeAbsorption, ...
         r.LightSources, r.VolumeIllumination, ...
         single([r.FactorEmission, r.FactorReflection, r.FactorAbsorption]), single(r.ElementSizeUm), ...
         uint64(resolution), single(flip(r.RotationMatrix)), single([0, r.FocalLength, r.DistanceToObject]), ...
         single(r.OpacityThreshold), single(r.Color)};
    if ~any([islogical(r.VolumeGradientX), islogical(r.VolumeGradientY), islogical(r.VolumeGradientZ)])
        c = [c, {r.VolumeGradientX, r.VolumeGradientY, r.VolumeGradientZ}];  % gradient lookup
    end
    cells{i} = c;
end
views = volumeRender('render_channels', cells, stereo, single(base));
stamp = timestamp;
for i = 1:n
    renderers{i}.TimeLastMemSync = stamp;
end
if ~stereo
    image = sum(views, 4);
    return;
end
leftImage = sum(views(:, :, :, 1:2:end), 4);    % page (i-1)*2 + 1: channel i, left eye (-base)
rightImage = sum(views(:, :, :, 2:2:end), 4);
leftImage = imcrop(leftImage, [(delta + 1) 0 size(leftImage, 2) size(leftImage, 1)]);
rightImage = imcrop(rightImage, [0 0 (size(rightImage, 2) - delta) size(rightImage, 1)]);
if r1.StereoOutput == StereoRenderMode.RedCyan
    image = zeros([size(leftImage, 1), size(leftImage, 2), 3]);
    image(:, :, 1) = leftImage(:, :, 1);
    image(:, :, 2) = rightImage(:, :, 2);
    image(:, :, 3) = rightImage(:, :, 3);
else
    image = [leftImage, rightImage];
end
end
