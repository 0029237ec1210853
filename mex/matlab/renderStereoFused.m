function image = renderStereoFused(r)
% renderStereoFused  The stereo branch of VolumeRender.render in one MEX call.
%
%   image = renderStereoFused(r)   % r: a VolumeRender with CameraXOffset ~= 0
%
% VolumeRender.render (VolumeRender.m:264-307) renders a stereo pair as two 'render' calls at
% camera offsets +base and -base over a widened image, crops delta columns from each and combines
% them by r.StereoOutput.  This function issues the pair as one volumeRender('render_stereo', ...)
% call (vr_render_stereo: both eyes in one launch, each image bit-identical to its 'render' call)
% and does the same widening, cropping and combining, so its result equals r.render().
%
% A VolumeRender.m that wants the fused path replaces its two p_render calls by
%   [leftImage, rightImage] = fusedPair(this, base, resolution)
% with the body of the MEX call below; nothing else in the class changes.
if r.CameraXOffset == 0
    image = r.render();
    return;
end
base = r.CameraXOffset / 2;
fov = 2 * atan(1 / r.FocalLength);
delta = round((base * r.ImageResolution(2)) / (2 * r.FocalLength * tan(fov / 2)));
resolution = flip(r.ImageResolution) + [0, delta];

lookup = ~any([islogical(r.VolumeGradientX), islogical(r.VolumeGradientY), islogical(r.VolumeGradientZ)]);
if lookup && ~all([isa(r.VolumeGradientX, 'Volume'), isa(r.VolumeGradientY, 'Volume'), isa(r.VolumeGradientZ, 'Volume')])
    error('All gradient dimensions need to be set and of type Volume!');
end
if all([islogical(r.VolumeReflection), islogical(r.VolumeAbsorption), islogical(r.VolumeEmission)])
    error('Not all volumes are properly set!');
end
r.syncVolumes();

factors = single([r.FactorEmission, r.FactorReflection, r.FactorAbsorption]);
props = single([0, r.FocalLength, r.DistanceToObject]);   % the x offset is the MEX's +-base
% the gradient volumes (lookup) reach the device through syncVolumes; 'render' does not read them
[leftImage, rightImage] = volumeRender('render_stereo', r.objectHandle, r.LightSources, ...
    r.VolumeIllumination, factors, single(r.ElementSizeUm), uint64(resolution), ...
    single(flip(r.RotationMatrix)), props, single(r.OpacityThreshold), single(r.Color), single(base));

leftImage = imcrop(leftImage, [(delta + 1) 0 size(leftImage, 2) size(leftImage, 1)]);
rightImage = imcrop(rightImage, [0 0 (size(rightImage, 2) - delta) size(rightImage, 1)]);
if r.StereoOutput == StereoRenderMode.RedCyan
    image = zeros([size(leftImage, 1), size(leftImage, 2), 3]);
    image(:, :, 1) = leftImage(:, :, 1);
    image(:, :, 2) = rightImage(:, :, 2);
    image(:, :, 3) = rightImage(:, :, 3);
else  % StereoRenderMode.LeftRightHorizontal
    image = [leftImage, rightImage];
end
end
