"""ctypes mirrors of the C structs (layouts of /root/reference/structures.py:6-106,
byte-identical to include/photohive_dsp.h), plus the new phd_config."""
import ctypes
from ctypes import POINTER, Structure, c_double, c_float, c_int, c_uint

Pixel = c_double


class Sharpnesses(Structure):
    _fields_ = [("N", c_int), ("sharpness", POINTER(Pixel))]


class Blur_Vector(Structure):
    _fields_ = [("angle", c_int), ("magnitude", c_float)]


class Blur_Vector_Group(Structure):
    _fields_ = [("len_vectors", c_int), ("blur_vectors", POINTER(Blur_Vector))]


class Pixel_HSV(Structure):
    _fields_ = [("parent_id", c_int), ("h", c_double), ("s", c_double), ("v", c_double)]


class Image_RGB(Structure):
    # c_uint as in the reference binding (structures.py:36-37); same size as C int
    _fields_ = [("height", c_uint), ("width", c_uint),
                ("r", POINTER(c_double)), ("g", POINTER(c_double)), ("b", POINTER(c_double))]


class Image_PGM(Structure):
    _fields_ = [("height", c_uint), ("width", c_uint), ("data", POINTER(c_double))]


class Color_Palette(Structure):
    _fields_ = [("N", c_int), ("averages", POINTER(Pixel_HSV)), ("percentages", POINTER(c_double))]


class RGB_Statistics(Structure):
    _fields_ = [("Br", c_double), ("Bg", c_double), ("Bb", c_double),
                ("Cr", c_double), ("Cg", c_double), ("Cb", c_double)]


class Crop_Boundaries(Structure):
    _fields_ = [("N", c_int), ("top", POINTER(c_int)), ("bottom", POINTER(c_int)),
                ("left", POINTER(c_int)), ("right", POINTER(c_int))]


class Blur_Profile(Structure):
    _fields_ = [("num_angle_bins", c_int), ("num_radius_bins", c_int),
                ("angle_bin_size", c_int), ("radius_bin_size", c_int),
                ("bins", POINTER(POINTER(c_double)))]

    def get_bin_values(self):
        return [[self.bins[i][j] for j in range(self.num_radius_bins)]
                for i in range(self.num_angle_bins)]


class Full_Report_Data(Structure):
    _fields_ = [("rgb_stats", POINTER(RGB_Statistics)), ("color_palette", POINTER(Color_Palette)),
                ("blur_profile", POINTER(Blur_Profile)), ("blur_vectors", POINTER(Blur_Vector_Group)),
                ("average_saturation", c_double), ("sharpness", POINTER(Sharpnesses))]


class PhdConfig(Structure):
    """The 16 scalar get_report hyper-parameters (include/photohive_dsp.h: phd_config)."""
    _fields_ = [("h_partitions", c_int), ("s_partitions", c_int), ("v_partitions", c_int),
                ("black_thresh", c_double), ("gray_thresh", c_double), ("coverage_thresh", c_double),
                ("linked_list_size", c_int), ("downsample_rate", c_int),
                ("radius_partitions", c_int), ("angle_partitions", c_int),
                ("quantity_weight", c_float), ("saturation_value_weight", c_float),
                ("fft_streak_thresh", c_double), ("magnitude_thresh", c_double),
                ("blur_cutoff_ratio_denom", c_int)]
