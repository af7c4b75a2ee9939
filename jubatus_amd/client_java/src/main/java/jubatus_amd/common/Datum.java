// Datum of the generated Java clients (jenerator -l java).
//
// Reference: jubatus/client/common/datum.hpp; wire form
// [string_values, num_values, binary_values], each a list of [key, value].
package jubatus_amd.common;

import java.util.ArrayList;
import java.util.List;

import org.msgpack.annotation.Message;

@Message
public class Datum {
  @Message
  public static class StringValue {
    public String key;
    public String value;
    public StringValue() {}
    public StringValue(String key, String value) {
      this.key = key;
      this.value = value;
    }
  }

  @Message
  public static class NumValue {
    public String key;
    public double value;
    public NumValue() {}
    public NumValue(String key, double value) {
      this.key = key;
      this.value = value;
    }
  }

  @Message
  public static class BinaryValue {
    public String key;
    public byte[] value;
    public BinaryValue() {}
    public BinaryValue(String key, byte[] value) {
      this.key = key;
      this.value = value;
    }
  }

  public List<StringValue> stringValues = new ArrayList<StringValue>();
  public List<NumValue> numValues = new ArrayList<NumValue>();
  public List<BinaryValue> binaryValues = new ArrayList<BinaryValue>();

  public Datum addString(String key, String value) {
    stringValues.add(new StringValue(key, value));
    return this;
  }

  public Datum addNumber(String key, double value) {
    numValues.add(new NumValue(key, value));
    return this;
  }

  public Datum addBinary(String key, byte[] value) {
    binaryValues.add(new BinaryValue(key, value));
    return this;
  }
}
